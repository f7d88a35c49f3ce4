#!/bin/bash
# blocks per match workgroup (ZT_DF_SUPER; streams identical): bench per setting
set -e
mkdir -p gpurun_out/r04sup
for k in 4 8 16 2 4; do
  ZT_DF_SUPER=$k timeout -k 10 300 python bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-api > gpurun_out/r04sup/bench_$k.log 2>&1
  echo "[super $k] $(tail -1 gpurun_out/r04sup/bench_$k.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["deflate_pipeline_ms"], d["match_kernel_ms"], d["ratio"])')"
done
