#!/bin/bash
# Round-3 end measurement on one MI355X, two gpurun calls:
#   A: GPU tests, smoke, PMC counters of the timed sources for the three workloads (bench, head4096 =
#      config 4, batch10 = config 5; profiles/counters_<workload>.json), the three bench lines
#   B: rocprofv3 kernel trace of the bench command, the batched bench pair's per-rank time at
#      N = 1, 2, 4, 8 on one device and head's own 8-way shard shape
#   gpurun -- bash tools/gpu_r03final.sh <tag> A|B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
R=$PWD
export TMPDIR=/tmp
T=${1:-r03final}
PART=${2:-A}
mkdir -p gpurun_out
run() {   # run <name> <seconds> <cmd...>: output to gpurun_out/${T}_<name>.log, stop on failure
    local name=$1 secs=$2; shift 2
    timeout -k 10 "$secs" "$@" > gpurun_out/${T}_${name}.log 2>&1
    local rc=$?
    echo "$name rc=$rc"; tail -c 300 gpurun_out/${T}_${name}.log | tail -1
    [ $rc -eq 0 ] || exit $rc
}
if [ "$PART" = A ]; then
    run pytest 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
    run smoke 120 python -c "import __graft_entry__ as g; g.smoke()"
    for W in bench head4096 batch10; do
        run counters_$W 600 python3 -u tools/collect_counters.py --workload $W --frames 8 \
            --out gpurun_out/${T}_counters_${W}.json --work gpurun_out/${T}_pmc
        cp gpurun_out/${T}_counters_${W}.json profiles/counters_${W}.json
    done
    run bench 300 python -u bench.py
    run bench_head4096 300 python -u bench.py --workload head4096 --no-end-to-end --no-moving-camera
    run bench_batch10 300 python -u bench.py --workload batch10 --no-end-to-end --no-moving-camera
    exit 0
fi
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${T}_trace -o run -- \
    python3 $R/bench.py --no-cpu-baseline --no-end-to-end --no-moving-camera \
    > $R/gpurun_out/${T}_bench_under_rocprof.json 2> $R/gpurun_out/${T}_trace.err
rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
cd $R
run shard_bench 300 python -u tools/shard_scaling.py --steady --batch --scenes 1 8 --out ${T}_shard_scaling_bench 0
run shard_head 500 python -u tools/shard_scaling.py --steady --scenes 4 --frame 4096 4096 16 \
    --out ${T}_shard_scaling_head 0
