# round-6 GPU session steps: bash tools/gpu_r06.sh TAG STEP [STEP ...]
#   tests    the wide-section / shard / batch / records GPU tests
#   gpu      the whole -m gpu suite
#   scale    tools/shard_scaling.py --steady --batch --overlap, scenes 1 8, LDS tier (default) and
#            the lane tier (RT_WH_LDS=0)
#   bench    bench.py at the driver's defaults
# Every step runs under its own time limit; the first failing step ends the call.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=$1; shift
run() {
    local name=$1 secs=$2; shift 2
    echo "[$(date +%T)] $name ..."
    timeout -k 10 "$secs" "$@" > gpurun_out/${T}_${name}.log 2>&1
    local rc=$?
    echo "[$(date +%T)] $name rc=$rc"
    [ $rc -eq 0 ] || { tail -20 gpurun_out/${T}_${name}.log; exit $rc; }
}
PYT="python -u -m pytest -x -v --timeout 200 --timeout-method thread"
for step in "$@"; do
    case $step in
    tests) run tests 700 $PYT tests/test_gpu_parity.py tests/test_gpu_overlap.py tests/test_gpu_views.py -m gpu \
               -k "tiers_agree or shard_hits_rank_of_8 or wide_heavy or batch_bench_pair or shard_partition_dense or tunables_read_once or head_4096x4096x16_eight or plan_race or moving_camera" ;;
    # the plan-race tests against the library built without HfCtx::fence: they must FAIL (recorded, not fatal)
    nofence) echo "[$(date +%T)] nofence ..."
             timeout -k 10 300 env RT_TRACER_LIB=librt_tracer_nofence.so python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_gpu_overlap.py -m gpu -k plan_race \
                 > gpurun_out/${T}_nofence.log 2>&1
             rc=$?; echo "[$(date +%T)] nofence rc=$rc (expected: 1, the tests fail without the fence)"
             [ $rc -le 1 ] || exit $rc ;;
    records) run records 600 $PYT tests/test_gpu_records.py tests/test_gpu_overlap.py tests/test_gpu_views.py -m gpu ;;
    gpu) run gpu 1100 $PYT tests -m gpu ;;
    scale) run scale_lds 400 python3 -u tools/shard_scaling.py --steady --batch --overlap --scenes 1 8 --out ${T}_scale_lds 0
           run scale_lanes 400 env RT_WH_LDS=0 RT_WH_BETA16=16 python3 -u tools/shard_scaling.py --steady --batch --overlap --scenes 1 8 --out ${T}_scale_lanes 0 ;;
    split) for v in split2 split16 split32; do
               run split_$v 200 env RT_TRACER_LIB=librt_tracer_$v.so python3 -u tools/shard_scaling.py --steady --batch --overlap \
                   --scenes 1 8 --out ${T}_split_$v 0
           done
           run split_base 200 python3 -u tools/shard_scaling.py --steady --batch --overlap --scenes 1 8 --out ${T}_split_base 0
           for cfg in "40 24" "40 32" "32 20" "32 28"; do
               set -- $cfg
               run ab_$1_$2 200 env RT_WH_ALPHA16=$1 RT_WH_BETA16=$2 python3 -u tools/shard_scaling.py --steady --batch --overlap \
                   --scenes 1 8 --out ${T}_ab_$1_$2 0
           done ;;
    alpha8) for cfg in "40 24" "48 24" "48 32" "56 32" "64 32"; do
               set -- $cfg
               run a8_$1_$2 200 env RT_WH_ALPHA16=$1 RT_WH_BETA16=$2 python3 -u tools/shard_scaling.py --steady --batch --overlap \
                   --scenes 1 8 --out ${T}_a8_$1_$2 0
           done ;;
    first) run first_proxy 300 python3 -u tools/first_frame_probe.py --scenes 0 1 2 3 4 5 6 7 8 9 --reps 3 --out ${T}_first_proxy
           run first_noproxy 300 env RT_TRACER_LIB=librt_tracer_noproxy.so python3 -u tools/first_frame_probe.py --scenes 0 1 2 3 4 5 6 7 8 9 --reps 3 --out ${T}_first_noproxy ;;
    move) run move 300 python -u bench.py --steps 200 --warmup 100 --no-cpu-baseline --no-end-to-end --no-first-frame --no-legs
          run move_driver 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-end-to-end --no-first-frame --no-legs ;;
    bench) run bench 300 python -u bench.py
           run bench_driver 300 python -u bench.py --steps 20 --warmup 5 ;;
    race) run race_prod 200 python3 -u tools/plan_race_probe.py --out ${T}_race_prod
          run race_nofence 200 env RT_TRACER_LIB=librt_tracer_nofence.so python3 -u tools/plan_race_probe.py --out ${T}_race_nofence ;;
    waves) run waves_lanes 200 env RT_WH_LDS=0 python3 -u tools/batch_waves.py --out ${T}_waves_lanes
           for b in 16 24; do
               run waves_lds_$b 200 env RT_WH_BETA16=$b python3 -u tools/batch_waves.py --out ${T}_waves_lds_$b
           done ;;
    floor) for cfg in "0 16 100000" "0 16 50000" "0 16 25000" "14 16 100000" "14 16 50000" "14 16 25000" "14 24 50000" "14 24 25000"; do
               set -- $cfg
               run floor_$1_$2_$3 200 env RT_WH_LDS=$1 RT_WH_BETA16=$2 RT_HF_FLOOR=$3 python3 -u tools/shard_scaling.py \
                   --steady --batch --overlap --scenes 1 8 --out ${T}_floor_$1_$2_$3 0
           done ;;
    floor2) for cfg in "0 16 100000" "14 16 50000" "14 24 50000" "14 24 100000" "14 32 50000"; do
               set -- $cfg
               run floor2_$1_$2_$3 200 env RT_WH_LDS=$1 RT_WH_BETA16=$2 RT_HF_FLOOR=$3 python3 -u tools/shard_scaling.py \
                   --steady --batch --overlap --scenes 1 8 --out ${T}_floor2_$1_$2_$3 0
           done
           run waves2_lds 200 env RT_WH_BETA16=24 RT_HF_FLOOR=50000 python3 -u tools/batch_waves.py --out ${T}_waves2_lds ;;
    order) for cfg in "0 16 100000" "0 16 50000" "14 24 50000" "8 24 50000" "8 24 30000"; do
               set -- $cfg
               run order_$1_$2_$3 200 env RT_WH_LDS=$1 RT_WH_BETA16=$2 RT_HF_FLOOR=$3 python3 -u tools/shard_scaling.py \
                   --steady --batch --overlap --scenes 8 1 --out ${T}_order_$1_$2_$3 0
           done ;;
    queues) run q4_scale 200 python3 -u tools/shard_scaling.py --steady --batch --overlap --scenes 1 8 --out ${T}_q4_scale 0
            run q16_scale 200 env GPU_MAX_HW_QUEUES=16 python3 -u tools/shard_scaling.py --steady --batch --overlap --scenes 1 8 --out ${T}_q16_scale 0
            run q4_bench 300 python -u bench.py --steps 200 --warmup 100 --no-cpu-baseline --no-end-to-end --no-first-frame --no-moving-camera --no-legs
            run q16_bench 300 env GPU_MAX_HW_QUEUES=16 python -u bench.py --steps 200 --warmup 100 --no-cpu-baseline --no-end-to-end --no-first-frame --no-moving-camera --no-legs ;;
    raceq) run raceq_nofence 200 env GPU_MAX_HW_QUEUES=16 RT_TRACER_LIB=librt_tracer_nofence.so python3 -u tools/plan_race_probe.py --out ${T}_raceq_nofence ;;
    tiers) for cfg in "0 32 16" "14 32 8" "14 32 12" "14 32 16" "14 32 24" "14 48 16" "14 64 16"; do
               set -- $cfg
               run tiers_$1_$2_$3 200 env RT_WH_LDS=$1 RT_WH_ALPHA16=$2 RT_WH_BETA16=$3 python3 -u tools/shard_scaling.py \
                   --steady --batch --overlap --scenes 1 8 --out ${T}_tiers_$1_$2_$3 0
           done ;;
    grid) run grid 300 $PYT tests/test_gpu_grid.py -m gpu
          run grid_bench 200 python3 -u tools/grid_bench.py --out gpurun_out/${T}_grid_bench.json ;;
    center) for c in 0 1; do
               run first_c$c 300 env RT_HF_CENTER=$c python3 -u tools/first_frame_probe.py --scenes 0 1 2 3 4 5 6 7 8 9 --reps 3 --out ${T}_first_c$c
           done
           for c in 0 1 0 1; do
               run scale_c$c 300 env RT_HF_CENTER=$c python3 -u tools/shard_scaling.py --steady --batch --overlap --scenes 1 8 --out ${T}_scale_c$c 0
               run bench_c$c 300 env RT_HF_CENTER=$c python -u bench.py --steps 200 --warmup 100 --no-cpu-baseline --no-end-to-end --no-legs
               run b10_c$c 300 env RT_HF_CENTER=$c python -u bench.py --workload batch10 --steps 50 --warmup 20 --no-cpu-baseline --no-end-to-end --no-first-frame --no-moving-camera --no-legs
           done ;;
    n1lds) for m in 0 15; do
               run n1lds_$m 300 python3 -u tools/tunable_sweep.py --env KERNEL --values 0 0x200 --scenes 4 5 8 2 --ns 1 \
                   --per-scene --extra-env RT_WH_LDS=$m --out ${T}_n1lds_$m
           done ;;
    *) echo "unknown step $step"; exit 2 ;;
    esac
done
