#!/bin/bash
# XCD-balanced match super-chunk order: digests (identical) + kernel stats A/B.
set -e
mkdir -p gpurun_out/xcd
ZT_LIB=$PWD/zlib.ts_amd/build/var_ref/libzt.so timeout -k 10 300 python3 -u tools/df_digest.py mixed > gpurun_out/xcd/ref.log 2>&1
timeout -k 10 300 python3 -u tools/df_digest.py mixed > gpurun_out/xcd/new.log 2>&1
grep "^L6" gpurun_out/xcd/ref.log gpurun_out/xcd/new.log
bash tools/gpu_kab.sh xcd_kab ref=zlib.ts_amd/build/var_ref/libzt.so new=new ref2=zlib.ts_amd/build/var_ref/libzt.so new2=new 2>&1 | grep -E "==|match_kernel"
