#!/bin/bash
# level-6 chain key length 6 / 4 at shorter chains (ZT_DF_PARAMS = chain,nice,lazy,skip,klen,probe,good,opt): gate + bench
set -e
mkdir -p gpurun_out/r04klen
for ps in 16,128,1,128,6,16,16,1 12,128,1,128,6,16,16,1 20,128,1,128,6,16,16,1 16,128,1,128,4,16,16,1; do
  name=$(echo $ps | tr ',' '_')
  timeout -k 10 300 python tools/ratio_gate.py "$ps" > gpurun_out/r04klen/gate_$name.log 2>&1
  ZT_DF_PARAMS=$ps timeout -k 10 300 python bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-api > gpurun_out/r04klen/bench_$name.log 2>&1
  echo "[$ps] $(grep '\[' gpurun_out/r04klen/gate_$name.log | sed 's/.*\] //' | cut -c1-200) | bench $(tail -1 gpurun_out/r04klen/bench_$name.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["deflate_pipeline_ms"], d["match_kernel_ms"], d["ratio"])')"
done
