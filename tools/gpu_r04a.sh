#!/bin/bash
# Round-4 GPU session A: GPU tests (incl. the product-kernel records), smoke, the bench line at the
# driver's and the steady settings, the batched step's wave timelines at N = 1, 2, 4, 8 (rank 0),
# and an in-process A/B of this build against the round-3 library (no regression from the record
# plumbing).    gpurun -- bash tools/gpu_r04a.sh <tag>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
T=${1:-r04a}
mkdir -p gpurun_out
run() {   # run <name> <seconds> <cmd...>: output to gpurun_out/${T}_<name>.log, stop on failure
    local name=$1 secs=$2; shift 2
    timeout -k 10 "$secs" "$@" > gpurun_out/${T}_${name}.log 2>&1
    local rc=$?
    echo "$name rc=$rc"; tail -c 400 gpurun_out/${T}_${name}.log | tail -2
    [ $rc -eq 0 ] || exit $rc
}
run pytest 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread
run smoke 120 python -c "import __graft_entry__ as g; g.smoke()"
run bench_driver 300 python -u bench.py --steps 20 --warmup 5
run bench 300 python -u bench.py --no-cpu-baseline
for N in 8 2 4 1; do
    run waves_n$N 200 python -u tools/batch_waves.py --rank 0 --nranks $N --frames 40 --out ${T}_waves_n$N
done
run ab_r03 300 python -u tools/ab_libs.py --arm new=librt_tracer.so:0 --arm r03=librt_tracer_r03.so:0 \
    --scenes 1 8 5 4 --rounds 6
