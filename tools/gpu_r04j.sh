#!/bin/bash
# Round-4 GPU session J: issue priority for the heavy-first front's waves (RT_HF_PRIO) at
# N = 1, 2, 4, 8, and the rank-of-8 wave timeline with and without it.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
T=${1:-r04j}
mkdir -p gpurun_out
run() {
    local name=$1 secs=$2; shift 2
    timeout -k 10 "$secs" "$@" > gpurun_out/${T}_${name}.log 2>&1
    local rc=$?
    echo "$name rc=$rc"; tail -c 400 gpurun_out/${T}_${name}.log | tail -2
    [ $rc -eq 0 ] || exit $rc
}
run prio 600 python -u tools/tunable_sweep.py --env RT_HF_PRIO --values 0 1 3 5 7 --ns 1 2 4 8 --rounds 2 --out ${T}_prio_sweep
run waves0 120 python3 -u tools/batch_waves.py --rank 0 --nranks 8 --out ${T}_waves_n8_prio0
RT_HF_PRIO=3 run waves3 120 python3 -u tools/batch_waves.py --rank 0 --nranks 8 --out ${T}_waves_n8_prio3
RT_HF_PRIO=7 run waves7 120 python3 -u tools/batch_waves.py --rank 0 --nranks 8 --out ${T}_waves_n8_prio7
