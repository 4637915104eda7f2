#!/bin/bash
# Round-4 GPU session F: per-lane (librt_tracer.so) vs time-synchronised (librt_tracer_tsync.so)
# vs lock-step (librt_tracer_lockstep.so) box runs: frames A/B on all 10 scenes, per-wave work of
# the t-sync build.      gpurun -- bash tools/gpu_r04f.sh <tag>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
T=${1:-r04f}
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/ab_libs.py --arm lockstep=librt_tracer_lockstep.so:0 --arm lane=librt_tracer.so:0 \
    --arm tsync=librt_tracer_tsync.so:0 --scenes 1 8 5 4 0 2 3 6 7 9 > gpurun_out/${T}_ab.json 2> gpurun_out/${T}_ab.err || exit $?
RT_TRACER_LIB=librt_tracer_tsync.so timeout -k 10 200 python3 -u tools/wave_mix.py --scenes 5 8 1 4 2 --out ${T}_tsync > gpurun_out/${T}_tsync.json 2> gpurun_out/${T}_tsync.err || exit $?
cat gpurun_out/${T}_ab.json gpurun_out/${T}_tsync.json
