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
FF="python3 -u tools/first_frame_probe.py --scenes 1 8 --reps 2"
run ff_trace0 120 env RT_HOST_TRACE=1 RT_HF_PROXY=0 $FF --out ${T}_ff_trace0
run ff_trace1 120 env RT_HOST_TRACE=1 RT_HF_PROXY_CELLS=3 $FF --out ${T}_ff_trace1
