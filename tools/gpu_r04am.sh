#!/bin/bash
# L2 (TCC) hits and misses of the bench's launches: batched pair, batched config 5, config 5 per scene
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
T=${1:-r04am}
mkdir -p gpurun_out
timeout -k 10 330 python3 -u tools/collect_counters.py --workload bench --batch --frames 8 --sets tcc \
    --out gpurun_out/${T}_tcc_bench.json --work gpurun_out/${T}_pmc > gpurun_out/${T}_1.log 2>&1 || exit $?
timeout -k 10 330 python3 -u tools/collect_counters.py --workload batch10 --batch --frames 8 --sets tcc \
    --out gpurun_out/${T}_tcc_batch10.json --work gpurun_out/${T}_pmc > gpurun_out/${T}_2.log 2>&1 || exit $?
timeout -k 10 330 python3 -u tools/collect_counters.py --workload batch10 --frames 8 --sets tcc \
    --out gpurun_out/${T}_tcc_batch10_per_scene.json --work gpurun_out/${T}_pmc_ps > gpurun_out/${T}_3.log 2>&1 || exit $?
python3 - <<'PY'
import json
for n in ("bench", "batch10", "batch10_per_scene"):
    d = json.load(open(f"gpurun_out/r04am_tcc_{n}.json"))["scenes"]
    for k, v in d.items():
        h, m = v["TCC_HIT_sum"], v["TCC_MISS_sum"]
        print(n, k, int(h), int(m), round(m / max(1.0, h + m), 4))
PY
