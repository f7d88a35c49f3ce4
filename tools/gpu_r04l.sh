#!/bin/bash
# level-6 parameter frontier on the 16-window gate + the 1 GiB bench's match time
# (ZT_DF_PARAMS = chain,nice,lazy,skip,klen,probe,good,opt)
set -e
mkdir -p gpurun_out/r04l
for ps in ${PARAMS:-"28,128,1,128,8,16,16,1" "28,128,1,128,8,16,12,1" "28,128,1,128,8,16,10,1" "28,128,1,128,8,16,8,1" "30,128,1,128,8,16,10,1" "32,128,1,128,8,16,8,1" "26,128,1,128,8,16,20,1"}; do
  timeout -k 10 300 python tools/ratio_gate.py "$ps" > gpurun_out/r04l/gate_$ps.log 2>&1
  ZT_DF_PARAMS=$ps timeout -k 10 300 python bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-api > gpurun_out/r04l/bench_$ps.log 2>&1
  echo "$ps | $(grep '\[' gpurun_out/r04l/gate_$ps.log | sed 's/.*wordsalad/wordsalad/' | cut -c1-60) ... $(grep -o 'worst.*' gpurun_out/r04l/gate_$ps.log) | bench $(tail -1 gpurun_out/r04l/bench_$ps.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["match_kernel_ms"], d["ratio"])')"
done
