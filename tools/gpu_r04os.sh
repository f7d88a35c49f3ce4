#!/bin/bash
# optparse cut lengths tried (ZT_OP_SHORT: 3..N, then only the full match): ratio gate + bench
set -e
R=$GRAFT_REPO_ROOT; mkdir -p gpurun_out/r04os
for spec in base= os14=sw_os14 os12=sw_os12 os10=sw_os10 os8=sw_os8; do
  name=${spec%%=*}; v=${spec#*=}
  if [ -n "$v" ]; then export ZT_LIB=$R/zlib.ts_amd/build/$v/libzt.so; else unset ZT_LIB; fi
  timeout -k 10 300 python tools/ratio_gate.py > gpurun_out/r04os/gate_$name.log 2>&1
  timeout -k 10 300 python bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-api > gpurun_out/r04os/bench_$name.log 2>&1
  echo "[$name] $(grep '\[' gpurun_out/r04os/gate_$name.log | sed 's/.*\] //' | cut -c1-200) | bench $(tail -1 gpurun_out/r04os/bench_$name.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["deflate_pipeline_ms"], d["match_kernel_ms"], d["ratio"])')"
done
