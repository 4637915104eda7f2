#!/bin/bash
# Round-4 GPU session M: the drop-in delivered inline by the waiting thread (RTH_POOL=0) with one
# whole-frame launch and one copy (RTH_LAUNCHES=1): GPU tests, breakdown, A/B against the pool.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
T=${1:-r04m}
mkdir -p gpurun_out
run() {
    local name=$1 secs=$2; shift 2
    timeout -k 10 "$secs" "$@" > gpurun_out/${T}_${name}.log 2>&1
    local rc=$?
    echo "$name rc=$rc"; tail -c 600 gpurun_out/${T}_${name}.log | tail -3
    [ $rc -eq 0 ] || exit $rc
}
run pytest 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread
run breakdown 240 python3 -u tools/e2e_breakdown.py --threads 1 16
run e2e 400 python -u tools/e2e_ab.py --arm "inline=" --arm "pool=;RTH_POOL=1" --arm "pool3=;RTH_POOL=1;RTH_LAUNCHES=3" \
    --arm "inline3=;RTH_LAUNCHES=3" --rounds 3 --reps 15
run bench 200 python3 -u bench.py --no-cpu-baseline --no-moving-camera
