#!/bin/bash
# Round-4 GPU session P: the wide section on AUTO's box runs with per-lane jumps (RT_WIDE_BOX=1,
# default build) vs the octant cube walk (librt_tracer_wideoct.so): parity, the batched rank-of-N
# step, the wide threshold at N = 4 and 8, the rank-of-8 timeline.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
T=${1:-r04p}
mkdir -p gpurun_out
run() {
    local name=$1 secs=$2; shift 2
    timeout -k 10 "$secs" "$@" > gpurun_out/${T}_${name}.log 2>&1
    local rc=$?
    echo "$name rc=$rc"; tail -c 400 gpurun_out/${T}_${name}.log | tail -2
    [ $rc -eq 0 ] || exit $rc
}
run pytest 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "record or shard or batch or wide or rank"
run shard_box 300 python -u tools/shard_scaling.py --steady --batch --scenes 1 8 --out ${T}_shard_widebox 0
RT_TRACER_LIB=librt_tracer_wideoct.so run shard_oct 300 python -u tools/shard_scaling.py --steady --batch --scenes 1 8 --out ${T}_shard_wideoct 0
run alpha8 400 python -u tools/tunable_sweep.py --env RT_WH_ALPHA16 --values 32 24 20 16 --ns 8 --rounds 2 --out ${T}_alpha8
run waves 150 python3 -u tools/batch_waves.py --rank 0 --nranks 8 --out ${T}_waves_n8
