#!/bin/bash
# longer optparse cut lengths (ZT_OP_SHORT 18/20/24) traded against a shorter chain: gate + bench
set -e
R=$GRAFT_REPO_ROOT; mkdir -p gpurun_out/r04os4
for spec in os24:20=sw_os24 os24:18=sw_os24 os28:20=sw_os28 os28:18=sw_os28 os32:18=sw_os32 os32:16=sw_os32; do
  name=${spec%%=*}; v=${spec#*=}; ch=${name#*:}
  if [ -n "$v" ]; then export ZT_LIB=$R/zlib.ts_amd/build/$v/libzt.so; else unset ZT_LIB; fi
  ps="$ch,128,1,128,8,16,16,1"
  timeout -k 10 300 python tools/ratio_gate.py "$ps" > gpurun_out/r04os4/gate_$name.log 2>&1
  ZT_DF_PARAMS=$ps timeout -k 10 300 python bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-api > gpurun_out/r04os4/bench_$name.log 2>&1
  echo "[$name] $(grep '\[' gpurun_out/r04os4/gate_$name.log | sed 's/.*\] //' | cut -c1-200) | bench $(tail -1 gpurun_out/r04os4/bench_$name.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["deflate_pipeline_ms"], d["match_kernel_ms"], d["ratio"])')"
done
