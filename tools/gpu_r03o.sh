#!/bin/bash
# Round-3 GPU session O: GPU tests + smoke of the current build, the rank-of-2 wide threshold sweep
# (RT_WH_ALPHA16_N2), the default bench line, PMC counters of the bench workload and the bench line
# that grades them, the rocprofv3 kernel trace of the bench command, and the batched shard scaling
# of the bench pair and of head at 4096^2 x 16.  Stops at the first step that faults, aborts or
# times out.
#   gpurun -- bash tools/gpu_r03o.sh <tag>      (env: SWEEP=0 / COUNTERS=0 / TRACE=0 / SCALE=0 skip steps)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
R=$PWD
export TMPDIR=/tmp
T=${1:-r03o}
mkdir -p gpurun_out
run() {   # run <name> <seconds> <cmd...>: output to gpurun_out/${T}_<name>.log, stop on failure
    local name=$1 secs=$2; shift 2
    timeout -k 10 "$secs" "$@" > gpurun_out/${T}_${name}.log 2>&1
    local rc=$?
    echo "$name rc=$rc"; tail -c 300 gpurun_out/${T}_${name}.log | tail -2
    [ $rc -eq 0 ] || exit $rc
}
run pytest 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
run smoke 120 python -c "import __graft_entry__ as g; g.smoke()"
if [ "${SWEEP:-1}" = 1 ]; then
    run alpha_n2 400 python -u tools/tunable_sweep.py --env RT_WH_ALPHA16_N2 --values 16 32 24 12 --ns 2 --rounds 4 \
        --out ${T}_alpha_n2_sweep
fi
run bench 300 python -u bench.py
if [ "${COUNTERS:-1}" = 1 ]; then
    run counters 600 python3 -u tools/collect_counters.py --workload bench --out gpurun_out/${T}_counters_bench.json \
        --work gpurun_out/${T}_pmc
    cp gpurun_out/${T}_counters_bench.json profiles/counters_bench.json
    run bench_counted 300 python -u bench.py --no-end-to-end --no-moving-camera --no-cpu-baseline
fi
if [ "${TRACE:-1}" = 1 ]; then
    cd /tmp
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${T}_trace -o run -- \
        python3 $R/bench.py --no-cpu-baseline --no-end-to-end --no-moving-camera \
        > $R/gpurun_out/${T}_bench_under_rocprof.json 2> $R/gpurun_out/${T}_trace.err
    rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
    cd $R
fi
if [ "${SCALE:-1}" = 1 ]; then
    run shard_bench 300 python -u tools/shard_scaling.py --steady --batch --scenes 1 8 --out ${T}_shard_scaling_bench 0
    run shard_head 500 python -u tools/shard_scaling.py --steady --scenes 4 --frame 4096 4096 16 \
        --out ${T}_shard_scaling_head 0
fi
