#!/bin/bash
# Round-3 GPU session Q: what bounds a frame at one rank -- per-wave real-time timelines of killeroo
# and Cornell at N = 1 and killeroo's rank 0 of 8 (RT_KERNEL_FLAG_WAVE_CLOCK), and the wide section
# forced at one rank (RT_KERNEL_FLAG_WIDE_HEAVY) against AUTO.
#   gpurun -- bash tools/gpu_r03q.sh <tag>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
T=${1:-r03q}
mkdir -p gpurun_out
run() {   # run <name> <seconds> <cmd...>: output to gpurun_out/${T}_<name>.log, stop on failure
    local name=$1 secs=$2; shift 2
    timeout -k 10 "$secs" "$@" > gpurun_out/${T}_${name}.log 2>&1
    local rc=$?
    echo "$name rc=$rc"; tail -c 300 gpurun_out/${T}_${name}.log | tail -2
    [ $rc -eq 0 ] || exit $rc
}
run waves_s8_n1 120 python -u tools/shard_waves.py 8 0 1
run waves_s1_n1 120 python -u tools/shard_waves.py 1 0 1
run waves_s8_n8 120 python -u tools/shard_waves.py 8 0 8
run waves_s1_n8 120 python -u tools/shard_waves.py 1 0 8
run ab_wide_n1 300 python -u tools/ab_kernels.py --kernels 0 0x200 --scenes 8 1 5 --rounds 8
