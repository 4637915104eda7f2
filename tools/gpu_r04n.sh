#!/bin/bash
# Round-4 GPU session N: two records per per-lane list iteration (RT_LANE_PAIR) vs one.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
T=${1:-r04n}
mkdir -p gpurun_out
run() {
    local name=$1 secs=$2; shift 2
    timeout -k 10 "$secs" "$@" > gpurun_out/${T}_${name}.log 2>&1
    local rc=$?
    echo "$name rc=$rc"; tail -c 400 gpurun_out/${T}_${name}.log | tail -2
    [ $rc -eq 0 ] || exit $rc
}
run ab 400 python -u tools/ab_libs.py --arm nopair=librt_tracer_nopair.so:0 --arm pair=librt_tracer_pair.so:0 --scenes 1 8 5 4 0 2 3 6 7 9
RT_TRACER_LIB=librt_tracer_pair.so run shard_pair 300 python -u tools/shard_scaling.py --steady --batch --scenes 1 8 --out ${T}_shard_pair 0
RT_TRACER_LIB=librt_tracer_nopair.so run shard_nopair 300 python -u tools/shard_scaling.py --steady --batch --scenes 1 8 --out ${T}_shard_nopair 0
