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
B="python -u bench.py --no-cpu-baseline --no-end-to-end --no-first-frame --no-moving-camera"
run pytest 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread
run b 100 $B
run b2 100 $B --steps 20 --warmup 5
run c 150 $B --workload batch10
run ser 100 python3 -u tools/frame_series.py --steps 60 --burn 200 --out ${T}_ser
run ser2 100 python3 -u tools/frame_series.py --steps 60 --burn 200 --out ${T}_ser2
run sweep 300 python -u tools/tunable_sweep.py --env RT_HF_FLOOR --values 100000 --ns 1 2 4 8 --rounds 2 --out ${T}_sweep
