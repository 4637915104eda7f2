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
run ovt 300 python -u -m pytest tests/test_gpu_overlap.py -x -q --timeout 200 --timeout-method thread
run single 300 python3 -u tools/overlap_stress.py --reps 4 --steps 40
run single_nf 300 python3 -u tools/overlap_stress.py --reps 2 --steps 40 --no-flag
run batch 300 python3 -u tools/overlap_stress.py --batch --reps 6 --steps 40
