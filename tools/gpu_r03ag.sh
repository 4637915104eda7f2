#!/bin/bash
# Round-3 GPU session AG: the cooperative (ray, record) pair arm inside the batched step
# (RT_KERNEL_FLAG_COOP_PAIRS = 0x1000) against AUTO at N = 1, 2, 4, 8, with the frames and hit IDs
# of the coop batch at N = 2 checked against the reference's.
#   gpurun -- bash tools/gpu_r03ag.sh <tag>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
T=${1:-r03ag}
mkdir -p gpurun_out
run() {
    local name=$1 secs=$2; shift 2
    timeout -k 10 "$secs" "$@" > gpurun_out/${T}_${name}.log 2>&1
    local rc=$?
    echo "$name rc=$rc"; tail -c 400 gpurun_out/${T}_${name}.log | tail -1
    [ $rc -eq 0 ] || exit $rc
}
run exact 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread \
    -k "batch_bench_pair or coop"
run coop 500 python -u tools/tunable_sweep.py --env KERNEL --values 0 0x1000 --ns 1 2 4 8 --rounds 3 \
    --out ${T}_coop_batch
