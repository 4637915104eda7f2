#!/bin/bash
# bench.py A/B of two builds of librt_tracer.so (RT_TRACER_LIB), alternating, N=1:
#   bash tools/ab_libs_bench.sh <lib_a> <lib_b> [rounds]
set -o pipefail
for r in $(seq 1 ${3:-3}); do
for L in $1 $2; do
  RT_TRACER_LIB=$L timeout -k 10 200 python3 -u ${AB_CMD:-bench.py --no-cpu-baseline --no-end-to-end} > gpurun_out/abl_${L}_$r.json 2>/dev/null || exit $?
  echo $L $r $(tail -c 2000 gpurun_out/abl_${L}_$r.json | python3 -c "import sys,json;t=sys.stdin.read().strip().splitlines()[-1];print(json.loads(t)['ms_per_step'] if t.startswith('{') else t)")
done; done
