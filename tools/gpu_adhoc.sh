# ad-hoc GPU session; edited per experiment
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-adhoc}
timeout -k 10 200 python3 -u tools/stream_overlap.py > gpurun_out/${T}_streams.json 2> gpurun_out/${T}_streams.err
rc=$?; cat gpurun_out/${T}_streams.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-end-to-end > gpurun_out/${T}_bench_w5.json 2>&1 && timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-end-to-end --warmup 100 --steps 200 > gpurun_out/${T}_bench_w100.json 2>&1
rc=$?; cut -c1-330 gpurun_out/${T}_bench_w5.json gpurun_out/${T}_bench_w100.json; exit $rc
