#!/bin/bash
# Round-5 session: the segmented wide tier -- its GPU tests, the wide / batch / records tests it
# touches, then in-process A/Bs of the tier (RT_WH_SEG_MIN_RANKS 0 = off) and of the wide threshold
# with it on, at the bench pair's rank-of-4 / rank-of-8 batched step.
#   gpurun -- bash tools/gpu_seg.sh <tag> [tests|ab|all]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
T=${1:-seg}
PART=${2:-all}
mkdir -p gpurun_out
run() {
    local name=$1 secs=$2; shift 2
    timeout -k 10 "$secs" "$@" > gpurun_out/${T}_${name}.log 2>&1
    local rc=$?
    echo "$name rc=$rc"; tail -c 400 gpurun_out/${T}_${name}.log | tail -3
    [ $rc -eq 0 ] || exit $rc
}
if [ "$PART" = tests ] || [ "$PART" = all ]; then
    run seg_tests 600 python -u -m pytest tests/test_gpu_segments.py -x -v --timeout 200 --timeout-method thread
    run rec_tests 600 python -u -m pytest tests/test_gpu_records.py -x -q --timeout 200 --timeout-method thread -k "batch or rank_of_8"
    run wide_tests 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "wide or batch or shard or rank_of_8"
fi
if [ "$PART" = ab ] || [ "$PART" = all ]; then
    run ab_seg 600 python -u tools/tunable_sweep.py --env RT_WH_SEG_MIN_RANKS --values 0 4 --ns 4 8 --rounds 3 --out ${T}_ab_seg
    run ab_alpha 600 python -u tools/tunable_sweep.py --env RT_WH_ALPHA16 --values 32 24 16 12 --ns 8 --rounds 2 --out ${T}_ab_alpha
fi
