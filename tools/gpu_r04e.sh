#!/bin/bash
# Round-4 GPU session E: per-wave work (cycles, uniform records, lane iterations) of the per-lane
# box runs vs the lock-step build.     gpurun -- bash tools/gpu_r04e.sh <tag>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
T=${1:-r04e}
mkdir -p gpurun_out
timeout -k 10 200 python3 -u tools/wave_mix.py --scenes 5 8 1 4 2 --out ${T}_lane > gpurun_out/${T}_lane.json 2> gpurun_out/${T}_lane.err || exit $?
RT_TRACER_LIB=librt_tracer_lockstep.so timeout -k 10 200 python3 -u tools/wave_mix.py --scenes 5 8 1 4 2 --out ${T}_lock > gpurun_out/${T}_lock.json 2> gpurun_out/${T}_lock.err || exit $?
cat gpurun_out/${T}_lane.json gpurun_out/${T}_lock.json
