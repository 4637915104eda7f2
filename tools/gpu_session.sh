#!/bin/bash
# One GPU-box session: the GPU tests, an optional in-process A/B of this build against another,
# PMC counters of this build (profiles/counters_bench.json, keyed by the kernel-source hash), the bench
# line, and the rocprofv3 kernel-trace stats of the same bench command.  Stops at the first step
# that faults, aborts or times out.
#   gpurun -- bash tools/gpu_session.sh <tag> [lib_b]
#   env: TESTS=0 skips pytest, COUNTERS=0 skips the PMC passes, TRACE=0 skips the kernel trace,
#        BENCH_ARGS="..." extra bench.py arguments, E2E_AB=<libdir> A/B of the Framebuffer path
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
R=$PWD
export TMPDIR=/tmp
TAG=${1:-run}
LIBB=${2:-}
mkdir -p gpurun_out
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }   # 1 = test failures / assertion, no fault
if [ "${TESTS:-1}" = 1 ]; then
    timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
        > gpurun_out/${TAG}_pytest.log 2>&1
    rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/${TAG}_pytest.log
    ok $rc || exit $rc
fi
if [ -n "$LIBB" ]; then
    timeout -k 10 300 python -u tools/ab_libs.py --lib-b "$LIBB" --scenes 1 8 5 4 --rounds 6 \
        > gpurun_out/${TAG}_ab.json 2> gpurun_out/${TAG}_ab.err
    rc=$?; echo "ab rc=$rc"; cat gpurun_out/${TAG}_ab.json
    ok $rc || exit $rc
fi
if [ -n "${E2E_AB:-}" ]; then
    timeout -k 10 400 python3 -u tools/e2e_ab.py --arm new= --arm prev=$E2E_AB \
        > gpurun_out/${TAG}_e2e_ab.log 2>&1
    rc=$?; echo "e2e_ab rc=$rc"; tail -1 gpurun_out/${TAG}_e2e_ab.log
    ok $rc || exit $rc
fi
if [ "${COUNTERS:-1}" = 1 ]; then
    timeout -k 10 900 python3 -u tools/collect_counters.py --workload bench --out gpurun_out/${TAG}_counters.json \
        --work gpurun_out/${TAG}_pmc > gpurun_out/${TAG}_counters.log 2>&1
    rc=$?; echo "counters rc=$rc"; tail -2 gpurun_out/${TAG}_counters.log
    [ $rc -eq 0 ] || exit $rc
    cp gpurun_out/${TAG}_counters.json profiles/counters_bench.json
fi
timeout -k 10 300 python -u bench.py ${BENCH_ARGS:-} > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/${TAG}_bench.json
[ $rc -eq 0 ] || exit $rc
if [ "${TRACE:-1}" = 1 ]; then
    cd /tmp
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${TAG}_trace -o run -- \
        python3 $R/bench.py --no-cpu-baseline --no-end-to-end ${BENCH_ARGS:-} \
        > $R/gpurun_out/${TAG}_bench_under_rocprof.json 2> $R/gpurun_out/${TAG}_trace.err
    rc=$?; echo "trace rc=$rc"
    exit $rc
fi
