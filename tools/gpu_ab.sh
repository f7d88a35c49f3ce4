#!/bin/bash
# A/B of two libzt builds on deflate output digests and kernel times:
# zlib.ts_amd/build/ref/libzt.so (before) vs zlib.ts_amd/libzt.so (after).
#   usage: tools/gpu_ab.sh TAG [kinds...]
set -e
TAG=${1:-ab}; shift || true
mkdir -p gpurun_out
ZT_LIB=$PWD/zlib.ts_amd/build/ref/libzt.so timeout -k 10 300 python3 tools/df_digest.py "$@" > gpurun_out/${TAG}_ref.log 2>&1
timeout -k 10 300 python3 tools/df_digest.py "$@" > gpurun_out/${TAG}_new.log 2>&1
paste -d'|' <(grep ratio gpurun_out/${TAG}_ref.log) <(grep ratio gpurun_out/${TAG}_new.log | cut -c1-200)
