#!/bin/bash
# Stall / instruction-mix counters for the render kernel, one rocprofv3 --pmc pass per set
# (never combined with trace domains).  Usage: bash tools/gpu_counters.sh <tag> <kernel>...
set -u
TAG=$1; shift
R=$PWD
OUT=$R/gpurun_out/ctr_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
SETS=(
  "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVES"
  "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_SMEM"
  "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_THREAD_CYCLES_VALU"
  "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum"
  "TCP_TCC_READ_REQ_LATENCY_sum TCP_TCP_LATENCY_sum"
  "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INST_LEVEL_VMEM"
)
for K in "$@"; do
  i=0
  for S in "${SETS[@]}"; do
    timeout -k 10 240 rocprofv3 --pmc $S --output-format csv -d $OUT/k${K}_$i -o run -- \
        python3 $R/tools/prof_render.py --reps 4 --kernel $K > $OUT/k${K}_$i.log 2>&1
    rc=$?; echo "k$K set$i rc=$rc"
    [ $rc -ne 0 ] && [ $i -lt 3 ] && exit 1
    i=$((i+1))
  done
done
echo counters-done
