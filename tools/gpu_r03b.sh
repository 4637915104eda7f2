#!/bin/bash
# Round-3 GPU session B: GPU tests + smoke, the bench line, the A/Bs of this session's changes
# (the cooperative pair pass at 1 rank and per rank of N; the row-rotated shard deal against the
# plain t mod N build librt_tracer_rot0.so), PMC counters of the bench workload, the rocprofv3
# kernel trace of the bench command and head's own shard scaling.  Stops at the first step that
# faults, aborts or times out.
#   gpurun -- bash tools/gpu_r03b.sh <tag>
#   env: TESTS=0 / AB=0 / COUNTERS=0 / TRACE=0 / SCALE=0 skip those steps
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
R=$PWD
export TMPDIR=/tmp
T=${1:-r03i}
mkdir -p gpurun_out
run() {   # run <name> <seconds> <cmd...>: output to gpurun_out/${T}_<name>.log, stop on failure
    local name=$1 secs=$2; shift 2
    timeout -k 10 "$secs" "$@" > gpurun_out/${T}_${name}.log 2>&1
    local rc=$?
    echo "$name rc=$rc"; tail -c 600 gpurun_out/${T}_${name}.log | tail -3
    [ $rc -eq 0 ] || exit $rc
}
if [ "${TESTS:-1}" = 1 ]; then
    run pytest 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread
    run smoke 120 python -c "import __graft_entry__ as g; g.smoke()"
fi
run bench 300 python -u bench.py
if [ "${AB:-1}" = 1 ]; then
    run ab_coop 300 python -u tools/ab_kernels.py --kernels 0 0x1000 --scenes 1 8 5 4 --rounds 10
    run shard_coop 400 python -u tools/shard_scaling.py --steady --scenes 8 5 --out ${T}_shard_coop 0 0x1000
    run shard_rot3 300 python -u tools/shard_scaling.py --steady --batch --scenes 1 8 5 --out ${T}_shard_rot3 0
    RT_TRACER_LIB=librt_tracer_rot0.so run shard_rot0 300 python -u tools/shard_scaling.py --steady --batch \
        --scenes 1 8 5 --out ${T}_shard_rot0 0
fi
if [ "${COUNTERS:-1}" = 1 ]; then
    run counters 600 python3 -u tools/collect_counters.py --workload bench --out gpurun_out/${T}_counters_bench.json \
        --work gpurun_out/${T}_pmc
    cp gpurun_out/${T}_counters_bench.json profiles/counters_bench.json
    run bench_counted 300 python -u bench.py --no-end-to-end --no-moving-camera --no-cpu-baseline
fi
if [ "${TRACE:-1}" = 1 ]; then
    cd /tmp
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${T}_trace -o run -- \
        python3 $R/bench.py --no-cpu-baseline --no-end-to-end --no-moving-camera \
        > $R/gpurun_out/${T}_bench_under_rocprof.json 2> $R/gpurun_out/${T}_trace.err
    rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
    cd $R
fi
if [ "${SCALE:-1}" = 1 ]; then
    run shard_head 500 python -u tools/shard_scaling.py --steady --scenes 4 --frame 4096 4096 16 \
        --out ${T}_shard_scaling_head 0
fi
