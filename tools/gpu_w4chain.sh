#!/bin/bash
# 4-walk match variant (build/exp_w4): ratio gate and bench at shorter chains
set -e
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
VL=$R/zlib.ts_amd/build/exp_w4/libzt.so
ZT_LIB=$VL timeout -k 10 400 python3 tools/ratio_gate.py "24,128,1,128,8,16,16,1" "20,128,1,128,8,16,16,1" "16,128,1,128,8,16,16,1" > gpurun_out/${1}_gate.log 2>&1
grep '^\[' gpurun_out/${1}_gate.log
for c in 24 20; do
  ZT_DF_PARAMS="$c,128,1,128,8,16,16,1" ZT_LIB=$VL timeout -k 10 300 python bench.py --no-cpu-baseline --no-api > gpurun_out/${1}_bench_$c.log 2>&1
  echo "[chain $c] $(tail -n 1 gpurun_out/${1}_bench_$c.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print({k: d[k] for k in ["value","ms_per_step","match_kernel_ms","deflate_pipeline_ms","ratio"]})')"
done
