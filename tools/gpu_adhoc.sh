# ad-hoc GPU session; edited per experiment
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
R=$PWD
T=${1:-adhoc}
run() {
    local name=$1 secs=$2; shift 2
    timeout -k 10 "$secs" "$@" > gpurun_out/${T}_${name}.log 2>&1
    local rc=$?
    echo "$name rc=$rc"
    [ $rc -eq 0 ] || { tail -5 gpurun_out/${T}_${name}.log; exit $rc; }
}
run ovtests 500 python -u -m pytest tests/test_gpu_overlap.py -x -v --timeout 300 --timeout-method thread
run h 150 python -u bench.py --no-cpu-baseline --workload head4096 --no-end-to-end --no-moving-camera --batch off
run h_off 150 python -u bench.py --no-cpu-baseline --workload head4096 --no-end-to-end --no-moving-camera --batch off --overlap off
