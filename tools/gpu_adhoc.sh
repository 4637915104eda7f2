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
run probe 120 tools/probe/dispatch_probe 40000 2000 5000 10000 20000
run w8_o8 120 python3 -u tools/batch_waves.py --rank 0 --nranks 8 --out ${T}_w8_o8
run ab_o8 600 python -u tools/tunable_sweep.py --env RT_WG64_O8 --values 0 1 --ns 2 4 8 --rounds 3 --out ${T}_ab_o8
run ab_wide_policy 600 python -u tools/tunable_sweep.py --env RT_WG64_WIDE --values 10 14 --ns 4 --rounds 3 --out ${T}_ab_wide_policy
run ab_alpha 600 python -u tools/tunable_sweep.py --env RT_WH_ALPHA16 --values 32 28 24 20 --ns 8 --rounds 2 --out ${T}_ab_alpha
