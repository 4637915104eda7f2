#!/bin/bash
# One GPU-box session: the GPU tests, an in-process A/B of this build against a previous one,
# and the bench line.  Stops at the first step that faults, aborts or times out.
#   gpurun -- bash tools/gpu_session.sh <tag> [lib_b]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
TAG=${1:-run}
LIBB=${2:-}
mkdir -p gpurun_out
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }   # 1 = test failures / assertion, no fault
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
    > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/${TAG}_pytest.log
ok $rc || exit $rc
if [ -n "$LIBB" ]; then
    timeout -k 10 300 python -u tools/ab_libs.py --lib-b "$LIBB" --scenes 1 8 5 4 --rounds 6 \
        > gpurun_out/${TAG}_ab.json 2> gpurun_out/${TAG}_ab.err
    rc=$?; echo "ab rc=$rc"; cat gpurun_out/${TAG}_ab.json
    ok $rc || exit $rc
fi
timeout -k 10 300 python -u bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/${TAG}_bench.json
exit $rc
