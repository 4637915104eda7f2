#!/bin/bash
# Round-4 GPU session C: GPU tests (the drop-in now issues from the starting thread), drop-in A/B,
# counters of the batched step at N = 1, 2, 8 (resident wave slots), the fused / side-stream wide
# section at N = 2, 4, 8, the LDS_CELLS arm on all 10 scenes, config 5's compaction A/B with HBM
# bytes (COMPACT now walks AUTO's box runs).    gpurun -- bash tools/gpu_r04c.sh <tag>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
T=${1:-r04c}
mkdir -p gpurun_out
run() {
    local name=$1 secs=$2; shift 2
    timeout -k 10 "$secs" "$@" > gpurun_out/${T}_${name}.log 2>&1
    local rc=$?
    echo "$name rc=$rc"; tail -c 600 gpurun_out/${T}_${name}.log | tail -3
    [ $rc -eq 0 ] || exit $rc
}
run pytest 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "framebuffer or tiled or frame_host or record or batch"
run e2e 300 python -u tools/e2e_ab.py --arm "copy=;RTH_TILED=0" --arm "late=;RTH_ISSUE_EARLY=0" --arm "t1=;RTH_LAUNCHES=1" \
    --arm "t2=;RTH_LAUNCHES=2" --arm "t3=;RTH_LAUNCHES=3" --rounds 3 --reps 11
for N in 8 2 1; do
    run counters_n$N 300 python3 -u tools/collect_counters.py --workload bench --batch --rank 0 --nranks $N --frames 24 \
        --sets sq --out gpurun_out/${T}_counters_batch_n$N.json --work gpurun_out/${T}_pmc_n$N
done
run fused 400 python -u tools/tunable_sweep.py --env RT_WH_FUSED --values 1 0 --ns 2 4 8 --rounds 2 --out ${T}_fused_sweep
run lds 300 python -u tools/ab_kernels.py --kernels 0 0x80 --scenes 0 1 2 3 4 5 6 7 8 9 --rounds 5 --reps 4
run batch10 600 bash tools/batch10_profile.sh ${T} 0 3
