#!/bin/bash
# after ordering a one-rank batch heaviest first: the batched workloads' counters, then the bench lines
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
T=${1:-r04ap}
mkdir -p gpurun_out
run() {
    local name=$1 secs=$2; shift 2
    timeout -k 10 "$secs" "$@" > gpurun_out/${T}_${name}.log 2>&1
    local rc=$?
    echo "$name rc=$rc"; tail -c 300 gpurun_out/${T}_${name}.log | tail -2
    [ $rc -eq 0 ] || exit $rc
}
for W in bench batch10; do
    run counters_$W 330 python3 -u tools/collect_counters.py --workload $W --frames 8 --batch \
        --out gpurun_out/${T}_counters_${W}.json --work gpurun_out/${T}_pmc
done
cp gpurun_out/${T}_counters_bench.json profiles/counters_bench.json
cp gpurun_out/${T}_counters_batch10.json profiles/counters_batch10.json
run bench 300 python -u bench.py
run bench_batch10 300 python -u bench.py --workload batch10 --no-end-to-end --no-moving-camera
run bench_s20w5 150 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline
