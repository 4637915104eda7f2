#!/bin/bash
# Round-3 GPU session K: GPU tests of the box-run empty runs (RT_BOX_RUN), their in-process A/B
# against the octant cube words in blocks of 4 (librt_tracer_cube.so) and the round-2 per-step loop
# (librt_tracer_skip1.so), the bench line, the cooperative pair A/B at 1 rank and per rank of N, and
# the batched shard scaling of the bench pair.  Stops at the
# first step that faults, aborts or times out.
#   gpurun -- bash tools/gpu_r03k.sh <tag>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
T=${1:-r03k}
mkdir -p gpurun_out
run() {   # run <name> <seconds> <cmd...>: output to gpurun_out/${T}_<name>.log, stop on failure
    local name=$1 secs=$2; shift 2
    timeout -k 10 "$secs" "$@" > gpurun_out/${T}_${name}.log 2>&1
    local rc=$?
    echo "$name rc=$rc"; tail -c 400 gpurun_out/${T}_${name}.log | tail -2
    [ $rc -eq 0 ] || exit $rc
}
run pytest 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
run ab_runs 400 python -u tools/ab_libs.py --arm box=librt_tracer.so:0 --arm cube4=librt_tracer_cube.so:0 \
    --arm step=librt_tracer_skip1.so:0 --scenes 1 8 5 4 0 7 --rounds 12
run bench 300 python -u bench.py --no-end-to-end --no-cpu-baseline
run ab_coop 300 python -u tools/ab_kernels.py --kernels 0 0x1000 --scenes 1 8 5 4 --rounds 10
run shard_coop 400 python -u tools/shard_scaling.py --steady --scenes 8 5 --out ${T}_shard_coop 0 0x1000
run shard_batch 300 python -u tools/shard_scaling.py --steady --batch --scenes 1 8 --out ${T}_shard_batch 0
