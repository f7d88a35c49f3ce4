#!/bin/bash
# match kernel: hop / extend counts per generator (build/var_dfcount) and the
# level-6 parameter frontier (tools/gpu_r04l.sh)
set -e
mkdir -p gpurun_out/r04m
ZT_LIB=$GRAFT_REPO_ROOT/zlib.ts_amd/build/var_dfcount/libzt.so timeout -k 10 180 python3 tools/df_count.py wordsalad structured mixed > gpurun_out/r04m/df_count.log 2>&1
grep -v amdgpu gpurun_out/r04m/df_count.log
bash tools/gpu_r04l.sh
