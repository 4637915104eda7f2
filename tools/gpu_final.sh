#!/bin/bash
# End-of-round measurement on one MI355X, in two gpurun calls (each well under the call limit):
#   part A: GPU tests, PMC counters of the timed sources for the three workloads (written to
#           profiles/counters_<workload>.json on the box, merged back via gpurun_out/), and the
#           three bench lines (bench, head4096 = config 4, batch10 = config 5)
#   part B: rocprofv3 kernel trace of the bench command, the batch10 compaction A/B with its
#           FETCH/WRITE passes, per-rank shard scaling and the lone-heavy-wave probe
#   gpurun -- bash tools/gpu_final.sh <tag> A|B
# Stops at the first step that faults, aborts or times out.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
R=$PWD
export TMPDIR=/tmp
T=${1:-final}
PART=${2:-A}
mkdir -p gpurun_out
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
if [ "$PART" = A ]; then
    timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
        > gpurun_out/${T}_pytest.log 2>&1
    rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/${T}_pytest.log
    ok $rc || exit $rc
    for W in bench head4096 batch10; do
        timeout -k 10 600 python3 -u tools/collect_counters.py --workload $W --frames 8 \
            --out gpurun_out/${T}_counters_${W}.json --work gpurun_out/${T}_pmc > gpurun_out/${T}_counters_${W}.log 2>&1
        rc=$?; echo "counters $W rc=$rc"
        [ $rc -eq 0 ] || exit $rc
        cp gpurun_out/${T}_counters_${W}.json profiles/counters_${W}.json
    done
    timeout -k 10 300 python -u bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err
    rc=$?; echo "bench rc=$rc"; cut -c1-300 gpurun_out/${T}_bench.json
    [ $rc -eq 0 ] || exit $rc
    timeout -k 10 300 python -u bench.py --workload head4096 > gpurun_out/${T}_bench_head4096.json 2> gpurun_out/${T}_bench_head4096.err
    rc=$?; echo "head4096 rc=$rc"
    [ $rc -eq 0 ] || exit $rc
    timeout -k 10 300 python -u bench.py --workload batch10 > gpurun_out/${T}_bench_batch10.json 2> gpurun_out/${T}_bench_batch10.err
    rc=$?; echo "batch10 rc=$rc"
    exit $rc
fi
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${T}_trace -o run -- \
    python3 $R/bench.py --no-cpu-baseline --no-end-to-end > $R/gpurun_out/${T}_bench_under_rocprof.json 2> $R/gpurun_out/${T}_trace.err
rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
cd $R
timeout -k 10 600 bash tools/batch10_profile.sh $T 0 3 536870915 1073741827 > gpurun_out/${T}_batch10.log 2>&1
rc=$?; echo "batch10 profile rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u tools/shard_scaling.py --steady --batch 0 1 > gpurun_out/${T}_shard.log 2>&1
rc=$?; echo "shard rc=$rc"; tail -n1 gpurun_out/${T}_shard.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 -u tools/tail_probe.py 0 > gpurun_out/${T}_tail_probe.log 2>&1
rc=$?; echo "tail probe rc=$rc"; exit $rc
