#!/bin/bash
# one-byte chain filter (ZT_DF_F8) against the 4-byte one: streams identical, match time
set -e
R=$GRAFT_REPO_ROOT; mkdir -p gpurun_out/r04f8
for spec in base= f8=var_f8 base2= f82=var_f8; do
  name=${spec%%=*}; v=${spec#*=}
  if [ -n "$v" ]; then export ZT_LIB=$R/zlib.ts_amd/build/$v/libzt.so; else unset ZT_LIB; fi
  timeout -k 10 300 python bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-api > gpurun_out/r04f8/bench_$name.log 2>&1
  echo "[$name] bench $(tail -1 gpurun_out/r04f8/bench_$name.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["deflate_pipeline_ms"], d["match_kernel_ms"], d["ratio"])')"
done
