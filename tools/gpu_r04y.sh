#!/bin/bash
# Round-4 GPU session Y: the second wide tier's parity (default G = 4, and the G = 2 build) and its
# threshold sweep with 2 lanes per sample.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
T=${1:-r04y}
mkdir -p gpurun_out
run() {
    local name=$1 secs=$2; shift 2
    timeout -k 10 "$secs" "$@" > gpurun_out/${T}_${name}.log 2>&1
    local rc=$?
    echo "$name rc=$rc"; tail -c 300 gpurun_out/${T}_${name}.log | tail -2
    [ $rc -eq 0 ] || exit $rc
}
run test_t4 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k second_wide_tier
RT_TRACER_LIB=librt_tracer_t2.so run test_t2 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k second_wide_tier
RT_TRACER_LIB=librt_tracer_t2.so run beta_t2 500 python -u tools/tunable_sweep.py --env RT_WH_BETA16 --values 0 24 20 16 12 --ns 4 8 --rounds 2 --out ${T}_beta_t2
