#!/bin/bash
# 16-window ratio gate + match time for variant builds in zlib.ts_amd/build/exp_NAME.
#   usage: tools/gpu_variants_gate.sh TAG NAME...
TAG=$1; shift
mkdir -p gpurun_out
timeout -k 10 200 python3 tools/ratio_gate.py "" > gpurun_out/${TAG}_base.log 2>&1 && echo "base $(grep '^\[' gpurun_out/${TAG}_base.log)"
for v in "$@"; do
  ZT_LIB=$PWD/zlib.ts_amd/build/exp_$v/libzt.so timeout -k 10 200 python3 tools/ratio_gate.py "" > gpurun_out/${TAG}_$v.log 2>&1 || exit 1
  echo "$v $(grep '^\[' gpurun_out/${TAG}_$v.log)"
done
