#!/bin/bash
# Ratio gate + L6 digests for several libzt builds: tools/gpu_libs.sh TAG lib1 lib2 ...
set -e
TAG=$1; shift
mkdir -p gpurun_out
for L in "$@"; do
  echo "== $L"
  ZT_LIB=$PWD/$L timeout -k 10 300 python -u tools/ratio_gate.py "" > gpurun_out/${TAG}_gate.log 2>&1; grep level6 gpurun_out/${TAG}_gate.log
  ZT_LIB=$PWD/$L timeout -k 10 300 python3 tools/df_digest.py wordsalad xorshift32 structured mixed > gpurun_out/${TAG}_dig.log 2>&1; grep L6 gpurun_out/${TAG}_dig.log
done
