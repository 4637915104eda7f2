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
run ser 100 python3 -u tools/frame_series.py --steps 60 --burn 1500 --kernel-times --out ${T}_ser
run ser2 100 python3 -u tools/frame_series.py --steps 60 --burn 1500 --kernel-times --out ${T}_ser2
