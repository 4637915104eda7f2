#!/bin/bash
# Round-3 GPU session AC: the wide threshold at a rank of 4 with 256-lane and with one-wave
# workgroups.   gpurun -- bash tools/gpu_r03ac.sh <tag>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
T=${1:-r03ac}
mkdir -p gpurun_out
run() {
    local name=$1 secs=$2; shift 2
    timeout -k 10 "$secs" "$@" > gpurun_out/${T}_${name}.log 2>&1
    local rc=$?
    echo "$name rc=$rc"; tail -c 400 gpurun_out/${T}_${name}.log | tail -1
    [ $rc -eq 0 ] || exit $rc
}
run alpha_n4 300 python -u tools/tunable_sweep.py --env RT_WH_ALPHA16 --values 32 48 64 4000 --ns 4 --rounds 3 \
    --out ${T}_alpha_n4
run alpha_n4_w64 300 python -u tools/tunable_sweep.py --env RT_WH_ALPHA16 --values 32 48 64 4000 --ns 4 --rounds 3 \
    --extra-env RT_WG64_WIDE=14 --out ${T}_alpha_n4_w64
