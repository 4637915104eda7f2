#!/bin/bash
# Round-3 GPU session AB: GPU tests of the rank-count policy (fused wide section from 2 ranks,
# one-wave workgroups at 1, 2 and >= 8 ranks) and its sweep against 256-lane workgroups beside the
# section, then the default bench line and the N = 2 one-device rehearsal.
#   gpurun -- bash tools/gpu_r03ab.sh <tag>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
T=${1:-r03ab}
mkdir -p gpurun_out
run() {   # run <name> <seconds> <cmd...>: output to gpurun_out/${T}_<name>.log, stop on failure
    local name=$1 secs=$2; shift 2
    timeout -k 10 "$secs" "$@" > gpurun_out/${T}_${name}.log 2>&1
    local rc=$?
    echo "$name rc=$rc"; tail -c 400 gpurun_out/${T}_${name}.log | tail -1
    [ $rc -eq 0 ] || exit $rc
}
run pytest 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
run smoke 120 python -c "import __graft_entry__ as g; g.smoke()"
run policy 400 python -u tools/tunable_sweep.py --env RT_WG64_WIDE --values 10 0 --ns 2 4 8 --rounds 4 \
    --out ${T}_wg64_wide_policy
run bench 300 python -u bench.py --no-end-to-end --no-cpu-baseline
