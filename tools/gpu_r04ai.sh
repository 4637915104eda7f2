#!/bin/bash
# k_hf_plan with 8 blocks per thread: GPU tests, then the kernel trace of a 20 + 5 bench run (static + moving camera)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
R=$PWD
T=${1:-r04ai}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 \
    || { tail -30 gpurun_out/${T}_pytest.log; exit 1; }
tail -2 gpurun_out/${T}_pytest.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${T}_mc -o run -- \
    python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-end-to-end --no-first-frame > $R/gpurun_out/${T}_mc.log 2>&1 || exit $?
cut -c1-200 $R/gpurun_out/${T}_mc/run_kernel_stats.csv
cd $R
timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-end-to-end --no-first-frame > gpurun_out/${T}_bench.log 2>&1 || exit $?
python3 -c "
import json; l=[x for x in open('gpurun_out/${T}_bench.log') if x.startswith('{\"metric')][-1]; d=json.loads(l)
print('bench', d['value'], d['ms_per_step'], 'moving', d['moving_camera']['value'], d['moving_camera']['ms_per_step'], d['moving_camera']['vs_static'])"
