#!/bin/bash
# Round-3 GPU session AA: one-wave workgroups beside the wide section (RT_WG64_WIDE), the side-stream
# section at 2 ranks and the fused one from 2 ranks (RT_WH_FUSED_MIN_RANKS=2).
#   gpurun -- bash tools/gpu_r03aa.sh <tag>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
T=${1:-r03aa}
mkdir -p gpurun_out
run() {   # run <name> <seconds> <cmd...>: output to gpurun_out/${T}_<name>.log, stop on failure
    local name=$1 secs=$2; shift 2
    timeout -k 10 "$secs" "$@" > gpurun_out/${T}_${name}.log 2>&1
    local rc=$?
    echo "$name rc=$rc"; tail -c 400 gpurun_out/${T}_${name}.log | tail -1
    [ $rc -eq 0 ] || exit $rc
}
run wide_w64 400 python -u tools/tunable_sweep.py --env RT_WG64_WIDE --values 0 1 --ns 2 4 8 --rounds 3 \
    --out ${T}_wg64_wide_sweep
run fused2_w64 300 python -u tools/tunable_sweep.py --env RT_WG64_WIDE --values 0 1 --ns 2 --rounds 3 \
    --extra-env RT_WH_FUSED_MIN_RANKS=2 --out ${T}_wg64_wide_fused2_sweep
