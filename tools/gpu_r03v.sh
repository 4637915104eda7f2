set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
run() { local name=$1 secs=$2; shift 2; timeout -k 10 "$secs" "$@" > gpurun_out/r03v_${name}.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -1 gpurun_out/r03v_${name}.log | cut -c1-600; [ $rc -eq 0 ] || exit $rc; }
run main 400 python -u tools/launch_ab.py --values 0 2 3 --rounds 3 --out r03v_persist_main
RT_TRACER_LIB=librt_tracer_pqnowpe.so run nowpe 300 python -u tools/launch_ab.py --values 0 1 --rounds 2 --out r03v_persist_nowpe
RT_TRACER_LIB=librt_tracer_pqsub1.so run sub1 300 python -u tools/launch_ab.py --values 0 1 --rounds 2 --out r03v_persist_sub1
