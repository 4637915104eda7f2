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
run pytest 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread
run single 300 python3 -u tools/overlap_stress.py --reps 4 --steps 40
run batch 300 python3 -u tools/overlap_stress.py --batch --reps 6 --steps 40
run ser 100 python3 -u tools/frame_series.py --steps 60 --burn 1500 --out ${T}_ser
run bench 150 python -u bench.py --no-cpu-baseline --no-end-to-end --no-first-frame --no-moving-camera
run c 150 python -u bench.py --no-cpu-baseline --workload batch10 --no-moving-camera
run ov 300 python3 -u tools/overlap_probe.py --rounds 2 --out ${T}_ov
