#!/bin/bash
# Round-3 GPU session AD: the wide threshold around its default at ranks of 4 and 8.
#   gpurun -- bash tools/gpu_r03ad.sh <tag>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
T=${1:-r03ad}
mkdir -p gpurun_out
run() {
    local name=$1 secs=$2; shift 2
    timeout -k 10 "$secs" "$@" > gpurun_out/${T}_${name}.log 2>&1
    local rc=$?
    echo "$name rc=$rc"; tail -c 400 gpurun_out/${T}_${name}.log | tail -1
    [ $rc -eq 0 ] || exit $rc
}
run alpha 500 python -u tools/tunable_sweep.py --env RT_WH_ALPHA16 --values 32 20 24 28 36 40 --ns 4 8 --rounds 3 \
    --out ${T}_alpha_n4_n8
