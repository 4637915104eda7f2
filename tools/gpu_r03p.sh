#!/bin/bash
# Round-3 GPU session P: GPU tests + smoke of the grown boxes (RT_BOX_GROW: each cross side, then
# the major axis, grown one cell at a time while the box stays empty), their A/B against the
# ungrown boxes (librt_tracer_nogrow.so), the bench line, and BASELINE configs 4 (head at
# 4096^2 x 16) and 5 (all 10 scenes) through bench.py's workloads.
#   gpurun -- bash tools/gpu_r03p.sh <tag>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
T=${1:-r03p}
mkdir -p gpurun_out
run() {   # run <name> <seconds> <cmd...>: output to gpurun_out/${T}_<name>.log, stop on failure
    local name=$1 secs=$2; shift 2
    timeout -k 10 "$secs" "$@" > gpurun_out/${T}_${name}.log 2>&1
    local rc=$?
    echo "$name rc=$rc"; tail -c 300 gpurun_out/${T}_${name}.log | tail -2
    [ $rc -eq 0 ] || exit $rc
}
run pytest 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
run smoke 120 python -c "import __graft_entry__ as g; g.smoke()"
run ab_grow 400 python -u tools/ab_libs.py --arm grow=librt_tracer.so:0 --arm nogrow=librt_tracer_nogrow.so:0 \
    --scenes 1 8 5 4 0 7 2 9 --rounds 10
run bench 300 python -u bench.py --no-end-to-end --no-cpu-baseline
run head4096 400 python -u bench.py --workload head4096 --no-cpu-baseline --no-moving-camera
run batch10 400 python -u bench.py --workload batch10 --no-cpu-baseline --no-moving-camera
