#!/bin/bash
# Round-3 GPU session: tests, then bench A/B (batched step vs one launch per frame) and the
# per-rank shard scaling of the bench pair (per-scene launches and batched).  Stops at the first
# step that faults, aborts or times out.
#   gpurun -- bash tools/gpu_r03.sh <tag>      env: TESTS=0 skips pytest, SCALE=0 skips scaling
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
T=${1:-r03}
mkdir -p gpurun_out
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
if [ "${TESTS:-1}" = 1 ]; then
    timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
        > gpurun_out/${T}_pytest.log 2>&1
    rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/${T}_pytest.log
    ok $rc || exit $rc
    [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 300 python -u bench.py --no-cpu-baseline --batch on > gpurun_out/${T}_bench_batch.json 2> gpurun_out/${T}_bench_batch.err
rc=$?; echo "bench batch rc=$rc"; cut -c1-400 gpurun_out/${T}_bench_batch.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-end-to-end --batch off > gpurun_out/${T}_bench_nobatch.json 2> gpurun_out/${T}_bench_nobatch.err
rc=$?; echo "bench no-batch rc=$rc"; cut -c1-400 gpurun_out/${T}_bench_nobatch.json; [ $rc -eq 0 ] || exit $rc
if [ "${SCALE:-1}" = 1 ]; then
    timeout -k 10 400 python -u tools/shard_scaling.py --steady --batch --scenes 1 8 --out ${T}_shard_scaling 0 \
        > gpurun_out/${T}_shard.log 2>&1
    rc=$?; echo "shard rc=$rc"; tail -1 gpurun_out/${T}_shard.log; [ $rc -eq 0 ] || exit $rc
fi
