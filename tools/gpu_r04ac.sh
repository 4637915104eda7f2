#!/bin/bash
# batched launches of up to 6 frames (config 5 as 5 + 5): the batch tests, then config 5 and the bench pair
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
T=${1:-r04ac}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_records.py -k "batch or records" -x -q \
    --timeout 200 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 || { tail -20 gpurun_out/${T}_pytest.log; exit 1; }
tail -2 gpurun_out/${T}_pytest.log
for W in batch10 bench; do
  timeout -k 10 200 python -u bench.py --workload $W --no-cpu-baseline --no-end-to-end --no-moving-camera \
      --no-first-frame > gpurun_out/${T}_${W}.log 2>&1 || exit $?
  python3 -c "
import json; l=[x for x in open('gpurun_out/${T}_${W}.log') if x.startswith('{\"metric')][-1]; d=json.loads(l)
print('$W', d['value'], d['ms_per_step'], d['config']['launch'], d['roofline'].get('counters'))"
done
