set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 330 python3 -u tools/collect_counters.py --workload batch10 --frames 8 --sets sq --out gpurun_out/pos_counters_ps.json --work gpurun_out/pos_pmc_ps > gpurun_out/pos_counters_ps.log 2>&1
timeout -k 10 300 python3 tools/tunable_sweep.py --per-scene --rounds 2 --scenes 0 1 2 3 4 5 6 7 8 9 --ns 1 --env RT_HF_POS16 --values 0 16 --out sw_pos_f > gpurun_out/sw_pos_f.log 2>&1
