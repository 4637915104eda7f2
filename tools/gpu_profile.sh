#!/bin/bash
# One gpurun call worth of profiling: kernel trace + separate PMC passes (FETCH_SIZE and
# WRITE_SIZE cannot share a pass on gfx950; counters never combined with sys/runtime traces).
# Usage (on the GPU box, from the repo root):  bash tools/gpu_profile.sh <tag> [kernel]
set -u
TAG=${1:-r01}
K=${2:-0}
R=$PWD
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
run() {  # name, then rocprofv3 args
  local name=$1; shift
  timeout -k 10 240 rocprofv3 "$@" --output-format csv -d $OUT/$name -o run -- \
      python3 $R/tools/prof_render.py --reps 10 --kernel $K > $OUT/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"
  return $rc
}
timeout -k 10 120 rocprofv3 -L > $OUT/counters.txt 2>&1; echo "list rc=$?"
run trace --kernel-trace --stats || exit 1
run fetch --pmc FETCH_SIZE || exit 1
run write --pmc WRITE_SIZE || exit 1
run sq --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES || exit 1
run valu --pmc SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VALU SQ_THREAD_CYCLES_VALU || true
run l2 --pmc TCC_HIT_sum TCC_MISS_sum || true
echo profile-done
