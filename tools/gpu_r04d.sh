#!/bin/bash
# Round-4 GPU session D: per-lane box runs (RT_LANE_RUNS=1) -- the GPU suite, an interleaved A/B
# against the lock-step build (librt_tracer_lockstep.so, -DRT_LANE_RUNS=0) on all 10 scenes, and
# the bench step with each build.      gpurun -- bash tools/gpu_r04d.sh <tag>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
T=${1:-r04d}
mkdir -p gpurun_out
run() {
    local name=$1 secs=$2; shift 2
    timeout -k 10 "$secs" "$@" > gpurun_out/${T}_${name}.log 2>&1
    local rc=$?
    echo "$name rc=$rc"; tail -c 800 gpurun_out/${T}_${name}.log | tail -4
    [ $rc -eq 0 ] || exit $rc
}
run pytest 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread
run ab 300 python -u tools/ab_libs.py --arm lane=librt_tracer.so:0 --arm lockstep=librt_tracer_lockstep.so:0 \
    --scenes 1 8 5 4 0 2 3 6 7 9
run bench 300 bash tools/ab_libs_bench.sh librt_tracer.so librt_tracer_lockstep.so 2
