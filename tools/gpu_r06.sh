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
           run scale_lanes 400 env RT_WH_LDS=0 python3 -u tools/shard_scaling.py --steady --batch --overlap --scenes 1 8 --out ${T}_scale_lanes 0 ;;
    bench) run bench 300 python -u bench.py ;;
    race) run race_prod 200 python3 -u tools/plan_race_probe.py --out ${T}_race_prod
          run race_nofence 200 env RT_TRACER_LIB=librt_tracer_nofence.so python3 -u tools/plan_race_probe.py --out ${T}_race_nofence ;;
    alpha) for tier in 0 14; do for a in 8 16 24 32 48; do
               run alpha_${tier}_${a} 200 env RT_WH_LDS=$tier RT_WH_ALPHA16=$a python3 -u tools/shard_scaling.py --steady \
                   --scenes 8 --out ${T}_alpha_${tier}_${a} 0
           done; done ;;
    *) echo "unknown step $step"; exit 2 ;;
    esac
done
