#!/bin/bash
# config 5 batched (5 + 5, cost-ordered) at N = 1: heavy-first floor and the wide section, bench.py lines
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
T=${1:-r04ag}
WH=512
mkdir -p gpurun_out
one() {
  local tag=$1; shift
  env "$@" timeout -k 10 200 python -u bench.py --workload batch10 --no-cpu-baseline --no-end-to-end \
      --no-moving-camera --no-first-frame $KARG > gpurun_out/${T}_${tag}.log 2>&1 || exit $?
  python3 -c "
import json; l=[x for x in open('gpurun_out/${T}_${tag}.log') if x.startswith('{\"metric')][-1]; d=json.loads(l)
print('$tag', d['value'], d['ms_per_step'])"
}
for rep in 1 2; do
  KARG="" one base_$rep X=1
  KARG="" one floor50k_$rep RT_HF_FLOOR=50000
  KARG="" one floor200k_$rep RT_HF_FLOOR=200000
  KARG="--kernel $WH" one wide_$rep RT_WH_FUSED_MIN_RANKS=1
done
