# ad-hoc GPU session; edited per experiment
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-adhoc}
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "cull or crop or full_frame_1080p4 or small_frames or head or auto_equals" > gpurun_out/${T}_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/${T}_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u tools/ab_libs.py --arm cull=librt_tracer.so:0 --arm nocull=librt_tracer.so:512 --arm c24=librt_tracer_c24.so:0 --arm c64=librt_tracer_c64.so:0 --arm base=librt_tracer_nocull.so:0 --scenes 1 8 5 4 --rounds 6 > gpurun_out/${T}_ab.json 2> gpurun_out/${T}_ab.err
rc=$?; cat gpurun_out/${T}_ab.json; [ $rc -eq 0 ] || exit $rc
RT_TRACER_LIB=librt_tracer_c24.so timeout -k 10 200 python3 tools/tail_probe.py 0 > gpurun_out/${T}_tp.log 2>&1
rc=$?; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u tools/shard_scaling.py 0 > gpurun_out/${T}_shard.log 2>&1
rc=$?; tail -n1 gpurun_out/${T}_shard.log; exit $rc
