#!/bin/bash
# bench.py A/B of two builds of librt_tracer.so (RT_TRACER_LIB), alternating, N=1:
#   bash tools/ab_libs_bench.sh <lib_a> <lib_b> [rounds]
set -o pipefail
for r in $(seq 1 ${3:-3}); do
for L in $1 $2; do
  RT_TRACER_LIB=$L timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --no-end-to-end > gpurun_out/abl_${L}_$r.json 2>/dev/null || exit $?
  echo $L $r $(python3 -c "import json;d=json.load(open('gpurun_out/abl_${L}_$r.json'));print(d['ms_per_step'], {k:v['kernel_ms'] for k,v in d['per_scene'].items()})")
done; done
