#!/bin/bash
# Round-3 GPU session N: GPU tests + smoke of the quad-split resolve (RT_QUAD_RESOLVE), its A/B
# against the single-lane resolve (librt_tracer_q0.so), the bench line, and a sweep of the wide
# section's threshold (RT_WH_ALPHA16) at 2 and 4 ranks for the batched bench pair.
#   gpurun -- bash tools/gpu_r03n.sh <tag>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
T=${1:-r03n}
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
run ab_quad 300 python -u tools/ab_libs.py --arm quad=librt_tracer.so:0 --arm one=librt_tracer_q0.so:0 \
    --scenes 1 8 5 4 0 7 2 --rounds 10
run bench 300 python -u bench.py --no-end-to-end --no-cpu-baseline
run alpha 500 python -u tools/tunable_sweep.py --env RT_WH_ALPHA16 --values 32 16 8 4 --ns 2 4 --rounds 2 \
    --out ${T}_alpha_sweep
