#!/bin/bash
# Build libzt.so with extra compile flags into build/var_NAME/ (tuning experiments;
# load it with ZT_LIB=...).   usage: tools/build_variant.sh NAME FLAGS...
# build/var_* is listed in .gpurunignore: drop that line while sweeping variants on the GPU.
set -e
NAME=$1; shift
cd "$(dirname "$0")/../zlib.ts_amd"
OUT=build/${VAR_PREFIX:-var_}$NAME; mkdir -p $OUT
pids=()
for f in csrc/*.hip csrc/*.cpp; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wno-unused-function "$@" -c -o $OUT/$(basename $f).o $f &
  pids+=($!)
done
for p in "${pids[@]}"; do wait $p || { echo "build_variant: a compile failed" >&2; exit 1; }; done
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -shared -o $OUT/libzt.so $OUT/*.o
echo built $OUT/libzt.so
