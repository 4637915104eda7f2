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
B="python -u bench.py --no-cpu-baseline --no-end-to-end --no-first-frame"
run pytest 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread
run part 300 python3 -u tools/batch_partition.py --arms "5+5 lpt" "10 lpt" "10 natural" --rounds 6 --out ${T}_part
run part_f2k 300 env RT_HF_FRONT_MAX=2048 python3 -u tools/batch_partition.py --arms "5+5 lpt" "10 lpt" --rounds 6 --out ${T}_part_f2k
run part_f4k 300 env RT_HF_FRONT_MAX=4096 python3 -u tools/batch_partition.py --arms "5+5 lpt" "10 lpt" --rounds 6 --out ${T}_part_f4k
run b10 200 $B --workload batch10 --no-moving-camera
run bench 150 $B
