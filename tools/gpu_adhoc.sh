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
run serb 100 python3 -u tools/frame_series.py --steps 40 --batch --time-every 8 --out ${T}_serb
run serb2 100 python3 -u tools/frame_series.py --steps 40 --batch --time-every 8 --out ${T}_serb2
run b2 100 $B --steps 20 --warmup 5
run b3 100 $B --steps 20 --warmup 5
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/${T}_btrace -o run -- \
    python3 $R/bench.py --no-cpu-baseline --no-end-to-end --no-first-frame --no-moving-camera --steps 20 --warmup 5 > $R/gpurun_out/${T}_btrace.log 2>&1
echo "btrace rc=$?"
