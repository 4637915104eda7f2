#!/bin/bash
# heavy-first front cap (RT_HF_FRONT_MAX) on config 5, the bench pair, and a rank of 8 of the pair
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
T=${1:-r04al}
mkdir -p gpurun_out
one() {
  local tag=$1 W=$2; shift 2
  env "$@" timeout -k 10 200 python -u bench.py --workload $W --no-cpu-baseline --no-end-to-end \
      --no-moving-camera --no-first-frame > gpurun_out/${T}_${tag}.log 2>&1 || exit $?
  python3 -c "
import json; l=[x for x in open('gpurun_out/${T}_${tag}.log') if x.startswith('{\"metric')][-1]; d=json.loads(l)
print('$tag', d['value'], d['ms_per_step'])"
}
for rep in 1 2; do
  for F in 1024 2048 4096; do
    one b10_f${F}_$rep batch10 RT_HF_FRONT_MAX=$F
    one bench_f${F}_$rep bench RT_HF_FRONT_MAX=$F
  done
done
for F in 1024 2048; do
  RT_HF_FRONT_MAX=$F timeout -k 10 300 python -u tools/shard_scaling.py --steady --batch --scenes 1 8 \
      --out ${T}_n8_f$F 0 > gpurun_out/${T}_n8_f$F.log 2>&1 || exit $?
  tail -c 300 gpurun_out/${T}_n8_f$F.log; echo
done
