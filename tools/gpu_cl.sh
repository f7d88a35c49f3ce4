#!/bin/bash
# Link steps in flight per group (-DZT_CL_U) vs the in-tree build: digests
# (identical) and match times per corpus.
set -e
mkdir -p gpurun_out/cl
timeout -k 10 300 python3 -u tools/df_digest.py wordsalad xorshift32 structured mixed > gpurun_out/cl/base.log 2>&1
ZT_LIB=$PWD/zlib.ts_amd/build/var_cl16/libzt.so timeout -k 10 300 python3 -u tools/df_digest.py wordsalad xorshift32 structured mixed > gpurun_out/cl/cl16.log 2>&1
timeout -k 10 300 python3 -u tools/df_digest.py wordsalad xorshift32 structured mixed > gpurun_out/cl/base2.log 2>&1
for f in base cl16 base2; do echo "== $f"; grep "^L6" gpurun_out/cl/$f.log; done
