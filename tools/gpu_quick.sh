#!/bin/bash
# Quick GPU iteration: deflate parity tests, then match-kernel time and ratio
# per corpus (128 MiB each) at level 6.   usage: tools/gpu_quick.sh TAG [pytest -k expr]
set -e
TAG=${1:-q}; K=${2:-deflate}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$K" > gpurun_out/${TAG}_t.log 2>&1 || { tail -30 gpurun_out/${TAG}_t.log; exit 1; }
tail -1 gpurun_out/${TAG}_t.log
for k in wordsalad xorshift32 structured; do
  timeout -k 10 120 python3 tools/df_sweep.py $k 32,128,1,128,8,16,16,1 2>&1 | grep ratio
done | tee gpurun_out/${TAG}_sweep.log
