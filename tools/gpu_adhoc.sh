# ad-hoc GPU session; edited per experiment
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-adhoc}
timeout -k 10 600 python3 -u tools/shard_scaling.py 0x8C000040 0x90000040 0x98000040 0x90000000 > gpurun_out/${T}_shard_budgets.log 2>&1
rc=$?; tail -n1 gpurun_out/${T}_shard_budgets.log; exit $rc
