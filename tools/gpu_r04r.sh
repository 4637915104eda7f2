#!/bin/bash
# Round-4 GPU session R: wide thresholds with the box-run wide walk -- the second tier (RT_WH_BETA16,
# 4 lanes per sample) at N = 4 and 8, and alpha at N = 8.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
T=${1:-r04r}
mkdir -p gpurun_out
run() {
    local name=$1 secs=$2; shift 2
    timeout -k 10 "$secs" "$@" > gpurun_out/${T}_${name}.log 2>&1
    local rc=$?
    echo "$name rc=$rc"; tail -c 300 gpurun_out/${T}_${name}.log | tail -2
    [ $rc -eq 0 ] || exit $rc
}
run beta 500 python -u tools/tunable_sweep.py --env RT_WH_BETA16 --values 0 16 20 24 --ns 4 8 --rounds 2 --out ${T}_beta
run alpha 300 python -u tools/tunable_sweep.py --env RT_WH_ALPHA16 --values 32 28 36 --ns 8 --rounds 2 --out ${T}_alpha
