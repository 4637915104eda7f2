#!/bin/bash
# Builds a variant of librt_tracer.so with extra compile switches, e.g. the ordering race of DESIGN.md
# §4.21 made visible (no HfCtx::fence):
#   tools/build_variant.sh nofence -DRT_DEBUG_NO_PLAN_FENCE
#   -> cpp-11-ray-trace-march-framework_amd/librt_tracer_<name>.so  (load it with RT_TRACER_LIB=<that file>)
set -e
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
C="$ROOT/cpp-11-ray-trace-march-framework_amd/csrc"
NAME=$1; shift
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-slp-vectorize"
TMP=$(mktemp -d)
pids=()
for tu in rt_kernels rt_plan rt_tracer rt_grid_build; do
    /opt/rocm/bin/hipcc $FLAGS "$@" -DRT_SRC_HASH="\"variant-$NAME\"" -c -o "$TMP/$tu.o" "$C/$tu.hip" &
    pids+=($!)
done
for p in "${pids[@]}"; do wait "$p"; done
/opt/rocm/bin/hipcc $FLAGS -shared -o "$C/../librt_tracer_$NAME.so" "$TMP"/*.o
rm -rf "$TMP"
echo "built librt_tracer_$NAME.so"
