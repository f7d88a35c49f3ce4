#!/bin/bash
# Checksum kernel variants (zlib.ts_amd/build/var_NAME/libzt.so, "base" = in-tree):
# correctness on odd sizes / offsets against zlib, then 1 GiB timings.
#   usage: tools/gpu_ck_variants.sh NAME...
set -e
R=$PWD
for v in "$@"; do
  lib=$R/zlib.ts_amd/libzt.so; [ $v = base ] || lib=$R/zlib.ts_amd/build/var_$v/libzt.so
  ZT_LIB=$lib timeout -k 10 120 python3 tools/ck_check.py 2>&1 | grep -v amdgpu.ids
  ZT_LIB=$lib timeout -k 10 120 python3 tools/ck_split.py 2>&1 | grep -v amdgpu.ids
done
