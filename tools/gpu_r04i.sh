#!/bin/bash
# Round-4 GPU session I: batched rank-of-N step, approach box runs (default) vs lock-step build.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
T=${1:-r04i}
mkdir -p gpurun_out
run() {
    local name=$1 secs=$2; shift 2
    timeout -k 10 "$secs" "$@" > gpurun_out/${T}_${name}.log 2>&1
    local rc=$?
    echo "$name rc=$rc"; tail -c 400 gpurun_out/${T}_${name}.log | tail -2
    [ $rc -eq 0 ] || exit $rc
}
run shard_approach 300 python -u tools/shard_scaling.py --steady --batch --scenes 1 8 --out ${T}_shard_approach 0
RT_TRACER_LIB=librt_tracer_lockstep.so run shard_lockstep 300 python -u tools/shard_scaling.py --steady --batch --scenes 1 8 --out ${T}_shard_lockstep 0
run shard_approach2 300 python -u tools/shard_scaling.py --steady --batch --scenes 1 8 --out ${T}_shard_approach2 0
