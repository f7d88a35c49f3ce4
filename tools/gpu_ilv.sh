#!/bin/bash
# Interleaved super-steps (-DZT_DF_ILV=F) vs the in-tree build: deflate
# digests (must be identical) and match / pipeline times per corpus.
set -e
mkdir -p gpurun_out/ilv
timeout -k 10 300 python3 -u tools/df_digest.py > gpurun_out/ilv/base.log 2>&1
for f in 2 4 8 16; do
  ZT_LIB=$PWD/zlib.ts_amd/build/var_ilv$f/libzt.so timeout -k 10 300 python3 -u tools/df_digest.py > gpurun_out/ilv/ilv$f.log 2>&1
done
for f in base ilv2 ilv4 ilv8 ilv16; do echo "== $f"; grep "^L6" gpurun_out/ilv/$f.log; done
