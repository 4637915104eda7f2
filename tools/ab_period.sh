set -o pipefail
for r in 1 2 3; do
for L in librt_tracer.so librt_tracer_p8.so librt_tracer_p16.so; do
  RT_TRACER_LIB=$L timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --no-end-to-end > gpurun_out/abp_${L}_$r.json 2>/dev/null || exit $?
  echo $L $r $(python3 -c "import json;d=json.load(open('gpurun_out/abp_${L}_$r.json'));print(d['ms_per_step'], {k:v['kernel_ms'] for k,v in d['per_scene'].items()})")
done; done
