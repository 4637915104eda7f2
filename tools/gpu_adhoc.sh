# ad-hoc GPU session; edited per experiment
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-adhoc}
run() {
    local name=$1 secs=$2; shift 2
    timeout -k 10 "$secs" "$@" > gpurun_out/${T}_${name}.log 2>&1
    local rc=$?
    echo "$name rc=$rc"
    [ $rc -eq 0 ] || { tail -5 gpurun_out/${T}_${name}.log; exit $rc; }
}
run ab_front 400 python -u tools/tunable_sweep.py --env RT_HF_FRONT_DIV --values 8 4 2 --ns 1 2 4 8 --rounds 2 --extra-env RT_HF_FRONT_MAX=4096 --out ${T}_ab_front
run ab_front1024 300 python -u tools/tunable_sweep.py --env RT_HF_FRONT_DIV --values 8 4 2 --ns 2 4 8 --rounds 2 --out ${T}_ab_front1024
run ab_shift 300 python -u tools/tunable_sweep.py --env RT_HF_SHIFT --values 2 3 --ns 1 2 4 8 --rounds 2 --out ${T}_ab_shift
