#!/bin/bash
# Builds an A/B variant of librt_tracer.so with build switches (rt_tracer.hip: RT_HF, RT_TB,
# RT_TDOT, RT_NO_LATE_PARAMS):  tools/build_variant.sh <name> -DRT_TB=0 ...
#   -> cpp-11-ray-trace-march-framework_amd/librt_tracer_<name>.so  (for tools/ab_libs.py)
set -e
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
C="$ROOT/cpp-11-ray-trace-march-framework_amd/csrc"
NAME=$1; shift
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-slp-vectorize"
TMP=$(mktemp -d)
/opt/rocm/bin/hipcc $FLAGS "$@" -c -o "$TMP/rt_tracer.o" "$C/rt_tracer.hip"
make -s -C "$C" rt_grid_build.o
/opt/rocm/bin/hipcc $FLAGS -shared -o "$C/../librt_tracer_$NAME.so" "$TMP/rt_tracer.o" "$C/rt_grid_build.o"
rm -rf "$TMP"
echo "built librt_tracer_$NAME.so"
