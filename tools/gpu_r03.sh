#!/bin/bash
# Round-3 GPU session: GPU tests + smoke, PMC counters of the bench workload, the bench line, the
# rocprofv3 kernel trace of the same bench command, and the per-rank shard scaling of the bench
# pair (per-scene launches and the batched step) and of head at 4096^2 x 16 (config 4).  Stops at
# the first step that faults, aborts or times out.
#   gpurun -- bash tools/gpu_r03.sh <tag>
#   env: TESTS=0 skips pytest + smoke, COUNTERS=0 the PMC passes, TRACE=0 the kernel trace,
#        SCALE=0 the shard scaling, BENCH_ARGS extra bench.py arguments
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
R=$PWD
export TMPDIR=/tmp
T=${1:-r03}
mkdir -p gpurun_out
if [ "${TESTS:-1}" = 1 ]; then
    timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
        > gpurun_out/${T}_pytest.log 2>&1
    rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/${T}_pytest.log
    [ $rc -eq 0 ] || exit $rc
    timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1
    rc=$?; echo "smoke rc=$rc"; [ $rc -eq 0 ] || exit $rc
fi
if [ "${COUNTERS:-1}" = 1 ]; then
    timeout -k 10 600 python3 -u tools/collect_counters.py --workload bench --out gpurun_out/${T}_counters_bench.json \
        --work gpurun_out/${T}_pmc > gpurun_out/${T}_counters.log 2>&1
    rc=$?; echo "counters rc=$rc"; [ $rc -eq 0 ] || exit $rc
    cp gpurun_out/${T}_counters_bench.json profiles/counters_bench.json
fi
timeout -k 10 300 python -u bench.py ${BENCH_ARGS:-} > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err
rc=$?; echo "bench rc=$rc"; cut -c1-300 gpurun_out/${T}_bench.json; [ $rc -eq 0 ] || exit $rc
if [ "${TRACE:-1}" = 1 ]; then
    cd /tmp
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${T}_trace -o run -- \
        python3 $R/bench.py --no-cpu-baseline --no-end-to-end --no-moving-camera ${BENCH_ARGS:-} \
        > $R/gpurun_out/${T}_bench_under_rocprof.json 2> $R/gpurun_out/${T}_trace.err
    rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
    cd $R
fi
if [ "${SCALE:-1}" = 1 ]; then
    timeout -k 10 400 python -u tools/shard_scaling.py --steady --batch --scenes 1 8 --out ${T}_shard_scaling_bench 0 \
        > gpurun_out/${T}_shard_bench.log 2>&1
    rc=$?; echo "shard bench rc=$rc"; tail -1 gpurun_out/${T}_shard_bench.log; [ $rc -eq 0 ] || exit $rc
    timeout -k 10 500 python -u tools/shard_scaling.py --steady --scenes 4 --frame 4096 4096 16 \
        --out ${T}_shard_scaling_head 0 > gpurun_out/${T}_shard_head.log 2>&1
    rc=$?; echo "shard head rc=$rc"; tail -1 gpurun_out/${T}_shard_head.log; [ $rc -eq 0 ] || exit $rc
fi
