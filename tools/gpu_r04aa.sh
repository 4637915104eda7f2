#!/bin/bash
# Round-4 GPU session AA: branch-free DDA setup (default build) vs the branchy one
# (librt_tracer_divbr.so); parity of the default build (frames, records, custom views).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
T=${1:-r04aa}
mkdir -p gpurun_out
run() {
    local name=$1 secs=$2; shift 2
    timeout -k 10 "$secs" "$@" > gpurun_out/${T}_${name}.log 2>&1
    local rc=$?
    echo "$name rc=$rc"; tail -c 300 gpurun_out/${T}_${name}.log | tail -2
    [ $rc -eq 0 ] || exit $rc
}
run pytest 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
run ab 400 python -u tools/ab_libs.py --arm divbr=librt_tracer_divbr.so:0 --arm flat=librt_tracer.so:0 --scenes 1 8 5 4 0 2 3 6 7 9
