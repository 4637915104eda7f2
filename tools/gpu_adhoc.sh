# ad-hoc GPU session (A/B of builds + PMC passes); edited per experiment
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-adhoc}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/${T}_pytest.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 400 python3 -u tools/ab_libs.py --arm main=librt_tracer.so:0 --arm prev=librt_tracer_prev.so:0 --scenes 1 8 5 4 --rounds 6 > gpurun_out/${T}_ab.json 2> gpurun_out/${T}_ab.err
rc=$?; cat gpurun_out/${T}_ab.json; [ $rc -eq 0 ] || exit $rc
SCENES="1 8" timeout -k 10 600 bash tools/pmc_ab.sh $T librt_tracer.so:0 librt_tracer_prev.so:0 > gpurun_out/${T}_pmc.log 2>&1
rc=$?; tail -1 gpurun_out/${T}_pmc.log; exit $rc
