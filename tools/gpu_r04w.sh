#!/bin/bash
# Round-4 GPU session W: the early re-planned heavy-first order (frames 2, 4, 8 measured) from a
# cold start and at the driver's 20 + 5 bench settings; the rank-of-8 timeline with the second
# wide tier on; the drop-in with two row-band launches whose bands take the heavy-first order.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
T=${1:-r04w}
mkdir -p gpurun_out
run() {
    local name=$1 secs=$2; shift 2
    timeout -k 10 "$secs" "$@" > gpurun_out/${T}_${name}.log 2>&1
    local rc=$?
    echo "$name rc=$rc"; tail -c 300 gpurun_out/${T}_${name}.log | tail -2
    [ $rc -eq 0 ] || exit $rc
}
run series_burn 100 python3 -u tools/frame_series.py --steps 60 --burn 1500 --out ${T}_series_burn
run series 100 python3 -u tools/frame_series.py --steps 60 --out ${T}_series
for i in 1 2 3; do
    run b20_$i 120 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-end-to-end --no-moving-camera --no-first-frame
done
RT_WH_BETA16=24 run waves_beta24 150 python3 -u tools/batch_waves.py --rank 0 --nranks 8 --out ${T}_waves_beta24
run e2e 400 python -u tools/e2e_ab.py --arm "l1=" --arm "l2=;RTH_LAUNCHES=2" --arm "l2hf=;RTH_LAUNCHES=2;RT_HF_MIN_BLOCKS=2048" \
    --arm "l1hf=;RT_HF_MIN_BLOCKS=2048" --rounds 3 --reps 15
