#!/bin/bash
# PMC counters of the render kernel for several builds / scenes, one rocprofv3 --pmc pass per
# counter set (never combined with trace domains):
#   bash tools/pmc_ab.sh <tag> "<lib>:<kernel>" ... ; summary: python3 tools/pmc_summary.py gpurun_out/pmc_<tag>
set -u
TAG=$1; shift
R=$PWD
OUT=$R/gpurun_out/pmc_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
SETS=(
  "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVES SQ_BUSY_CYCLES"
  "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_INSTS_LDS"
  "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_MISC SQ_THREAD_CYCLES_VALU"
)
for ARM in "$@"; do
  LIB=${ARM%%:*}; K=${ARM##*:}
  for SC in ${SCENES:-1 8}; do
    i=0
    for S in "${SETS[@]}"; do
      D=$OUT/${LIB%.so}_k${K}_s${SC}_$i
      timeout -k 10 120 rocprofv3 --pmc $S --output-format csv -d $D -o run -- \
          python3 $R/tools/render_loop.py --lib $LIB --scene $SC --frames 6 --kernel $K > $D.log 2>&1
      rc=$?; echo "$LIB k$K s$SC set$i rc=$rc"
      [ $rc -ne 0 ] && exit $rc
      i=$((i+1))
    done
  done
done
echo pmc-done
