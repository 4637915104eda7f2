#!/bin/bash
# Round-4 GPU session Q: whole-record loads in the per-lane list loop (RT_LANE_WHOLE=1, default
# build) vs the second half loaded inside the gate (librt_tracer_split.so).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
T=${1:-r04q}
mkdir -p gpurun_out
run() {
    local name=$1 secs=$2; shift 2
    timeout -k 10 "$secs" "$@" > gpurun_out/${T}_${name}.log 2>&1
    local rc=$?
    echo "$name rc=$rc"; tail -c 400 gpurun_out/${T}_${name}.log | tail -2
    [ $rc -eq 0 ] || exit $rc
}
run ab 400 python -u tools/ab_libs.py --arm split=librt_tracer_split.so:0 --arm whole=librt_tracer.so:0 --scenes 1 8 5 4 0 2 3 6 7 9
run shard_whole 300 python -u tools/shard_scaling.py --steady --batch --scenes 1 8 --out ${T}_shard_whole 0
RT_TRACER_LIB=librt_tracer_split.so run shard_split 300 python -u tools/shard_scaling.py --steady --batch --scenes 1 8 --out ${T}_shard_split 0
run waves 150 python3 -u tools/batch_waves.py --rank 0 --nranks 8 --out ${T}_waves_n8
