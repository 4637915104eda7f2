#!/bin/bash
# Round-4 GPU session H: approach modes -- 3 (approach, then lock-step), 4 (then time-synchronised),
# 5 (a new approach whenever the wave is inside boxes again) vs lock-step 0.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
T=${1:-r04h}
mkdir -p gpurun_out
run() {
    local name=$1 secs=$2; shift 2
    timeout -k 10 "$secs" "$@" > gpurun_out/${T}_${name}.log 2>&1
    local rc=$?
    echo "$name rc=$rc"; tail -c 600 gpurun_out/${T}_${name}.log | tail -3
    [ $rc -eq 0 ] || exit $rc
}
run ab 500 python -u tools/ab_libs.py --arm approach=librt_tracer_approach.so:0 --arm lockstep=librt_tracer_lockstep.so:0 \
    --arm appts=librt_tracer_appts.so:0 --arm reappr=librt_tracer_reappr.so:0 --scenes 1 8 5 4 0 2 3 6 7 9
