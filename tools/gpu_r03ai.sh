#!/bin/bash
# Round-3 GPU session AI: the N = 1 bench step as one batched launch vs one launch per frame,
# interleaved, 3 rounds.   gpurun -- bash tools/gpu_r03ai.sh <tag>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
T=${1:-r03ai}
mkdir -p gpurun_out
for r in 1 2 3; do
    for b in on off; do
        timeout -k 10 200 python -u bench.py --batch $b --no-end-to-end --no-cpu-baseline --no-moving-camera \
            > gpurun_out/${T}_${b}_$r.json 2> gpurun_out/${T}_${b}_$r.err
        rc=$?; [ $rc -eq 0 ] || { echo "bench $b $r rc=$rc"; exit $rc; }
        python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['kernel_ms_per_step'])" gpurun_out/${T}_${b}_$r.json $b
    done
done
