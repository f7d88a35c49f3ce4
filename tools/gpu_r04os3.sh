#!/bin/bash
# optparse cut lengths 18 / 20 at 4 waves per SIMD (spills) or 3 (none), chain 22: bench
set -e
R=$GRAFT_REPO_ROOT; mkdir -p gpurun_out/r04os3
export ZT_DF_PARAMS="22,128,1,128,8,16,16,1"
for spec in os20=sw_os20 os20m3=sw_os20m3 os18=sw_os18 os18m3=sw_os18m3 os20b=sw_os20 os20m3b=sw_os20m3; do
  name=${spec%%=*}; export ZT_LIB=$R/zlib.ts_amd/build/${spec#*=}/libzt.so
  timeout -k 10 300 python bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-api > gpurun_out/r04os3/bench_$name.log 2>&1
  echo "[$name] bench $(tail -1 gpurun_out/r04os3/bench_$name.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["deflate_pipeline_ms"], d["match_kernel_ms"], d["ratio"])')"
done
