#!/bin/bash
# Round-3 GPU session R: the wide section at ONE rank -- killeroo's heaviest waves (~1 M cycles)
# are about as long as its whole frame, so the frame may be critical-path bound there.  Forced
# (RT_KERNEL_FLAG_WIDE_HEAVY) against AUTO at several thresholds (RT_WH_ALPHA16, sixteenths of
# the span estimate), single launches and steady state (tools/steady_probe-style via shard_scaling
# at N = 1).
#   gpurun -- bash tools/gpu_r03r.sh <tag>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
T=${1:-r03r}
mkdir -p gpurun_out
run() {   # run <name> <seconds> <cmd...>: output to gpurun_out/${T}_<name>.log, stop on failure
    local name=$1 secs=$2; shift 2
    timeout -k 10 "$secs" "$@" > gpurun_out/${T}_${name}.log 2>&1
    local rc=$?
    echo "$name rc=$rc"; tail -c 300 gpurun_out/${T}_${name}.log | tail -2
    [ $rc -eq 0 ] || exit $rc
}
for a in 16 8 4 2; do
    RT_WH_ALPHA16=$a run ab_wide_a$a 200 python -u tools/ab_kernels.py --kernels 0 0x200 --scenes 8 5 1 --rounds 6
done
