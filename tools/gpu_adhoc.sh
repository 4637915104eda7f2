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
run bench 150 python -u bench.py --no-cpu-baseline
run bench_off 150 python -u bench.py --no-cpu-baseline --overlap off --no-end-to-end --no-moving-camera --no-first-frame
run b2 100 python -u bench.py --no-cpu-baseline --steps 20 --warmup 5
run c 150 python -u bench.py --no-cpu-baseline --workload batch10
run c_off 150 python -u bench.py --no-cpu-baseline --workload batch10 --overlap off
run h 150 python -u bench.py --no-cpu-baseline --workload head4096 --no-end-to-end --no-moving-camera
run shard 500 python -u tools/shard_scaling.py --steady --batch --overlap --scenes 1 8 --out ${T}_shard 0
