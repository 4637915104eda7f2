#!/bin/bash
# Round-4 GPU session G: AUTO's box-run modes -- approach + lock-step (librt_tracer.so,
# RT_LANE_RUNS=3) vs lock-step (0), per-lane (1), time-synchronised (2): GPU parity of the default
# build, frames A/B on all 10 scenes, per-wave work, the bench.     gpurun -- bash tools/gpu_r04g.sh <tag>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
T=${1:-r04g}
mkdir -p gpurun_out
run() {
    local name=$1 secs=$2; shift 2
    timeout -k 10 "$secs" "$@" > gpurun_out/${T}_${name}.log 2>&1
    local rc=$?
    echo "$name rc=$rc"; tail -c 600 gpurun_out/${T}_${name}.log | tail -3
    [ $rc -eq 0 ] || exit $rc
}
run pytest 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread
run ab 500 python -u tools/ab_libs.py --arm approach=librt_tracer.so:0 --arm lockstep=librt_tracer_lockstep.so:0 \
    --arm lane=librt_tracer_lane.so:0 --arm tsync=librt_tracer_tsync.so:0 --scenes 1 8 5 4 0 2 3 6 7 9
run mix 200 python3 -u tools/wave_mix.py --scenes 5 8 1 4 2 --out ${T}_approach
run bench 200 python3 -u bench.py --no-cpu-baseline --no-end-to-end
