#!/bin/bash
# BASELINE config 5: all 10 built-in scenes at 1920x1080x4spp as one batch, wavefront
# active-ray compaction A/B (RT_KERNEL_COMPACT vs AUTO), with rocprofv3 HBM traffic per launch.
# Usage (GPU box, repo root):  bash tools/batch10_profile.sh <tag> <kernel>...
# Each arm: in-process interleaved timing (ab_kernels.py) + separate FETCH_SIZE / WRITE_SIZE
# passes (never combined with trace domains; MI355X_MICROARCH.md §rocprofv3 PMC slots).
set -u
TAG=$1; shift
R=$PWD
OUT=$R/gpurun_out/batch10_$TAG
mkdir -p $OUT
timeout -k 10 300 python3 $R/tools/ab_kernels.py --kernels "$@" --scenes 0 1 2 3 4 5 6 7 8 9 \
    --rounds 5 --reps 4 > $OUT/ab.json 2> $OUT/ab.err || exit 1
echo "ab rc=0"
cd /tmp && export TMPDIR=/tmp
for K in "$@"; do
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 120 rocprofv3 --pmc $C --output-format csv -d $OUT/k${K}_$C -o run -- \
        python3 $R/tools/prof_render.py --reps 2 --kernel $K --scenes 0 1 2 3 4 5 6 7 8 9 \
        > $OUT/k${K}_$C.log 2>&1 || exit 1
    echo "k$K $C rc=0"
  done
done
echo batch10-done
