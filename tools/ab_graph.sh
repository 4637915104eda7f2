#!/bin/bash
# bench.py A/B: direct launches vs hipGraph replay (--graph), alternating, N=1
set -o pipefail
for r in 1 2 3; do
for A in direct graph; do
  X=""; [ $A = graph ] && X="--graph"
  timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --no-end-to-end $X > gpurun_out/abg_${A}_$r.json 2>/dev/null || exit $?
  echo $A $r $(python3 -c "import json;d=json.load(open('gpurun_out/abg_${A}_$r.json'));print(d['ms_per_step'], {k:v['kernel_ms'] for k,v in d['per_scene'].items()})")
done; done
