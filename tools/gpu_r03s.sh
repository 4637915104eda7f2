#!/bin/bash
# Round-3 GPU session S: the wide threshold (RT_WH_ALPHA16) at a rank of 8 for the batched bench pair
# (fused wide section), and per-rank timelines of the fused batch at N = 8.
#   gpurun -- bash tools/gpu_r03s.sh <tag>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
T=${1:-r03s}
mkdir -p gpurun_out
run() {   # run <name> <seconds> <cmd...>: output to gpurun_out/${T}_<name>.log, stop on failure
    local name=$1 secs=$2; shift 2
    timeout -k 10 "$secs" "$@" > gpurun_out/${T}_${name}.log 2>&1
    local rc=$?
    echo "$name rc=$rc"; tail -c 300 gpurun_out/${T}_${name}.log | tail -2
    [ $rc -eq 0 ] || exit $rc
}
run alpha_n8 500 python -u tools/tunable_sweep.py --env RT_WH_ALPHA16 --values 32 16 24 48 64 --ns 8 --rounds 3 \
    --out ${T}_alpha_n8_sweep
run floor_n8 400 python -u tools/tunable_sweep.py --env RT_WH_FLOOR --values 100000 50000 200000 --ns 8 --rounds 3 \
    --out ${T}_floor_n8_sweep
