#!/bin/bash
# Round-4 GPU session X: the next cell's word loaded before a non-empty cell's test
# (RT_CELL_PREFETCH=1, default build) vs not (librt_tracer_nopf.so).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
T=${1:-r04x}
mkdir -p gpurun_out
run() {
    local name=$1 secs=$2; shift 2
    timeout -k 10 "$secs" "$@" > gpurun_out/${T}_${name}.log 2>&1
    local rc=$?
    echo "$name rc=$rc"; tail -c 300 gpurun_out/${T}_${name}.log | tail -2
    [ $rc -eq 0 ] || exit $rc
}
run ab 400 python -u tools/ab_libs.py --arm nopf=librt_tracer_nopf.so:0 --arm pf=librt_tracer.so:0 --scenes 1 8 5 4 0 2 3 6 7 9
run shard_pf 300 python -u tools/shard_scaling.py --steady --batch --scenes 1 8 --out ${T}_shard_pf 0
RT_TRACER_LIB=librt_tracer_nopf.so run shard_nopf 300 python -u tools/shard_scaling.py --steady --batch --scenes 1 8 --out ${T}_shard_nopf 0
