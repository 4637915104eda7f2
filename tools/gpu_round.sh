#!/bin/bash
# Round end measurement on one MI355X, three gpurun calls:
#   A: GPU tests, smoke, PMC counters of the timed sources for the three workloads
#      (profiles/counters_<workload>.json via gpurun_out/)
#   B: the three bench lines (bench, head4096 = config 4, batch10 = config 5) and the driver's 20 + 5
#   C: rocprofv3 kernel trace of the bench command, per-rank shard scaling with the gather
#      rehearsal (bench pair, head), counters of a rank-of-8 batched step
#   gpurun -- bash tools/gpu_round.sh <tag> A|B|C
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
R=$PWD
export TMPDIR=/tmp
T=${1:-r04final}
PART=${2:-A}
mkdir -p gpurun_out
run() {
    local name=$1 secs=$2; shift 2
    timeout -k 10 "$secs" "$@" > gpurun_out/${T}_${name}.log 2>&1
    local rc=$?
    echo "$name rc=$rc"; tail -c 300 gpurun_out/${T}_${name}.log | tail -2
    [ $rc -eq 0 ] || exit $rc
}
if [ "$PART" = A ]; then
    run pytest 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread
    run smoke 120 python -c "import __graft_entry__ as g; g.smoke()"
    # bench.py renders a step's frames one launch each at N = 1 (overlapped; batched at N > 1): the
    # counters are per scene, summed per step by bench.py
    for W in bench batch10 head4096; do
        run counters_$W 330 python3 -u tools/collect_counters.py --workload $W --frames 8 \
            --out gpurun_out/${T}_counters_${W}.json --work gpurun_out/${T}_pmc
    done
    # per-scene launches of config 5 (each scene's own VALU issue fraction, not a bench input)
    run counters_batch10_per_scene 330 python3 -u tools/collect_counters.py --workload batch10 --frames 8 \
        --sets sq --out gpurun_out/${T}_counters_batch10_per_scene.json --work gpurun_out/${T}_pmc_ps
    exit 0
fi
if [ "$PART" = B ]; then
    run bench 300 python -u bench.py
    run bench_head4096 300 python -u bench.py --workload head4096 --no-end-to-end --no-moving-camera
    run bench_batch10 300 python -u bench.py --workload batch10 --no-end-to-end --no-moving-camera
    run bench_s20w5 150 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline
    run series_burn 100 python3 -u tools/frame_series.py --steps 60 --burn 1500 --out ${T}_series_burn
    exit 0
fi
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${T}_trace -o run -- \
    python3 $R/bench.py --no-cpu-baseline --no-end-to-end --no-moving-camera --no-first-frame \
    > $R/gpurun_out/${T}_bench_under_rocprof.json 2> $R/gpurun_out/${T}_trace.err
rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
cd $R
run shard_bench 500 python -u tools/shard_scaling.py --steady --batch --overlap --scenes 1 8 --out ${T}_shard_scaling_bench 0
run shard_head 500 python -u tools/shard_scaling.py --steady --scenes 4 --frame 4096 4096 16 --out ${T}_shard_scaling_head 0
run counters_n8 300 python3 -u tools/collect_counters.py --workload bench --batch --rank 0 --nranks 8 --frames 64 \
    --sets sq lat --out gpurun_out/${T}_counters_batch_n8.json --work gpurun_out/${T}_pmc_n8
