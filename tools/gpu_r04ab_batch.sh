#!/bin/bash
# A/B: one launch per frame vs batched launches (up to MAX_BATCH frames) at N = 1, bench pair and config 5
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
T=${1:-r04ab}
mkdir -p gpurun_out
for rep in 1 2; do
  for W in batch10 bench; do
    for B in off on; do
      timeout -k 10 200 python -u bench.py --workload $W --batch $B --steps 200 --warmup 100 --no-cpu-baseline \
          --no-end-to-end --no-moving-camera --no-first-frame > gpurun_out/${T}_${W}_${B}_${rep}.log 2>&1 || exit $?
      python3 -c "
import json; l=[x for x in open('gpurun_out/${T}_${W}_${B}_${rep}.log') if x.startswith('{\"metric')][-1]; d=json.loads(l)
print('$W $B $rep', d['value'], d['ms_per_step'], d.get('kernel_ms_per_step'))"
    done
  done
done
