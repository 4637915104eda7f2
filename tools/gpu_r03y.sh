#!/bin/bash
# Round-3 GPU session Y: GPU tests + smoke of the one-wave-workgroup build, the batched step with and
# without one-wave workgroups (RT_WG64) at N = 1, 2, 4, 8 ranks on one device, and the bench line.
#   gpurun -- bash tools/gpu_r03y.sh <tag>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
T=${1:-r03y}
mkdir -p gpurun_out
run() {   # run <name> <seconds> <cmd...>: output to gpurun_out/${T}_<name>.log, stop on failure
    local name=$1 secs=$2; shift 2
    timeout -k 10 "$secs" "$@" > gpurun_out/${T}_${name}.log 2>&1
    local rc=$?
    echo "$name rc=$rc"; tail -c 400 gpurun_out/${T}_${name}.log | tail -2
    [ $rc -eq 0 ] || exit $rc
}
run pytest 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
run smoke 120 python -c "import __graft_entry__ as g; g.smoke()"
run wg64_sweep 500 python -u tools/tunable_sweep.py --env RT_WG64 --values 1 0 --ns 1 2 4 8 --rounds 3 \
    --out ${T}_wg64_batch_sweep
run bench 300 python -u bench.py --no-end-to-end --no-cpu-baseline
