#!/bin/bash
# Round-4 GPU session B: GPU tests (records through the raw-record fixup, the zero-copy tiled
# drop-in, batch counters), the second wide tier's threshold swept at N = 2, 4, 8 for the batched
# bench pair, a rank-of-8 timeline with the tier, and the drop-in A/B (row-major + tile copies vs
# the tiled zero-copy frame at 1-4 row-band launches).    gpurun -- bash tools/gpu_r04b.sh <tag>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
T=${1:-r04b}
mkdir -p gpurun_out
run() {
    local name=$1 secs=$2; shift 2
    timeout -k 10 "$secs" "$@" > gpurun_out/${T}_${name}.log 2>&1
    local rc=$?
    echo "$name rc=$rc"; tail -c 600 gpurun_out/${T}_${name}.log | tail -3
    [ $rc -eq 0 ] || exit $rc
}
run pytest 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread
run e2e 300 python -u tools/e2e_ab.py --arm "copy=;RTH_TILED=0" --arm "t1=;RTH_LAUNCHES=1" --arm "t2=;RTH_LAUNCHES=2" \
    --arm "t3=;RTH_LAUNCHES=3" --arm "t4=;RTH_LAUNCHES=4" --rounds 3 --reps 11
run beta 600 python -u tools/tunable_sweep.py --env RT_WH_BETA16 --values 0 8 12 16 20 --ns 2 4 8 --rounds 2 \
    --out ${T}_beta_sweep
RT_WH_BETA16=12 run waves_n8_b12 200 python -u tools/batch_waves.py --rank 0 --nranks 8 --frames 40 --out ${T}_waves_n8_b12
RT_HF_FOLLOW=0 run mc_follow0 300 python -u bench.py --no-cpu-baseline --no-end-to-end --no-first-frame --steps 100 --warmup 20
RT_HF_FOLLOW=1 run mc_follow1 300 python -u bench.py --no-cpu-baseline --no-end-to-end --no-first-frame --steps 100 --warmup 20
