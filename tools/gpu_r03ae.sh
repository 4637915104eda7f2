#!/bin/bash
# Round-3 GPU session AE: heavy-first tunables at one rank on the one-wave-workgroup build (the bench
# pair, one launch per frame), and the rank-of-4 threshold check.
#   gpurun -- bash tools/gpu_r03ae.sh <tag>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
T=${1:-r03ae}
mkdir -p gpurun_out
run() {
    local name=$1 secs=$2; shift 2
    timeout -k 10 "$secs" "$@" > gpurun_out/${T}_${name}.log 2>&1
    local rc=$?
    echo "$name rc=$rc"; tail -c 300 gpurun_out/${T}_${name}.log | tail -1
    [ $rc -eq 0 ] || exit $rc
}
run hf_floor 400 python -u tools/tunable_sweep.py --env RT_HF_FLOOR --values 100000 50000 200000 400000 --ns 1 \
    --per-scene --rounds 3 --out ${T}_hf_floor_n1
run hf_off 300 python -u tools/tunable_sweep.py --env RT_HF_MIN_BLOCKS --values 4096 1000000000 --ns 1 \
    --per-scene --rounds 3 --out ${T}_hf_off_n1
run alpha_n4 300 python -u tools/tunable_sweep.py --env RT_WH_ALPHA16_N4 --values 28 32 --ns 4 --rounds 3 \
    --out ${T}_alpha_n4_check
