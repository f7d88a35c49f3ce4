#!/bin/bash
# level-6 parameter frontier on the 16-window gate + the 1 GiB bench's match time
# (ZT_DF_PARAMS = chain,nice,lazy,skip,klen,probe,good,opt)
set -e
mkdir -p gpurun_out/r04l
for ps in "28,128,1,128,8,16,16,1" "28,64,1,128,8,16,16,1" "28,32,1,128,8,16,16,1" "28,128,1,128,8,16,12,1" "32,48,1,128,8,16,16,1" "24,128,1,128,8,16,24,1"; do
  export ZT_DF_PARAMS=$ps
  timeout -k 10 300 python tools/ratio_gate.py > gpurun_out/r04l/gate_$ps.log 2>&1
  timeout -k 10 300 python bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-api > gpurun_out/r04l/bench_$ps.log 2>&1
  echo "$ps | $(grep '\[' gpurun_out/r04l/gate_$ps.log | sed 's/.*wordsalad/wordsalad/' | cut -c1-60) ... $(grep -o 'worst.*' gpurun_out/r04l/gate_$ps.log) | bench $(tail -1 gpurun_out/r04l/bench_$ps.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["match_kernel_ms"], d["ratio"])')"
done
