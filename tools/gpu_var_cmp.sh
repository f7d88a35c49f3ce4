#!/bin/bash
# Compare libzt variants (zlib.ts_amd/build/var_NAME/libzt.so; "base" = the
# in-tree build) on the 16-window ratio gate and 128 MiB match times.
#   usage: tools/gpu_var_cmp.sh TAG NAME... [-- PARAMS...]
TAG=$1; shift
names=(); params=("")
while [ $# -gt 0 ]; do [ "$1" = "--" ] && { shift; params=("$@"); break; }; names+=("$1"); shift; done
mkdir -p gpurun_out; R=$PWD
for nm in "${names[@]}"; do
  lib=$R/zlib.ts_amd/libzt.so; [ "$nm" = base ] || lib=$R/zlib.ts_amd/build/var_$nm/libzt.so
  echo "== $nm"
  ZT_LIB=$lib timeout -k 10 300 python3 tools/ratio_gate.py "${params[@]}" 2>&1 | grep -v amdgpu.ids || exit 1
  for k in wordsalad xorshift32 structured; do
    ZT_LIB=$lib timeout -k 10 120 python3 tools/df_sweep.py $k "${params[@]:-32,128,1,128,8,16,16,1}" 2>&1 | grep ratio || exit 1
  done
done 2>&1 | tee gpurun_out/${TAG}.log
