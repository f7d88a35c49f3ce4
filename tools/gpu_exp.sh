#!/bin/bash
# One-call experiment batch: 1 GiB bench lines (no CPU baseline / host API)
# for the in-tree build and variant builds / parameter sets.
#   usage: tools/gpu_exp.sh TAG "label|ZT_LIB-or-empty|ZT_DF_PARAMS-or-empty" ...
set -e
TAG=$1; shift
mkdir -p gpurun_out
for spec in "$@"; do
  IFS='|' read -r label lib params <<< "$spec"
  env ${lib:+ZT_LIB=$PWD/$lib} ${params:+ZT_DF_PARAMS=$params} timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-api > gpurun_out/${TAG}_${label}.log 2>&1
  echo "$label $(tail -1 gpurun_out/${TAG}_${label}.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["match_kernel_ms"], d["deflate_pipeline_ms"], d["inflate_kernel_ms"], d["ratio"], d.get("ratio_vs_ref"))')"
done
