#!/bin/bash
# ZT_DF_GREAT="len,hops": walks of positions with a long carried match cut
# to a few hops -- 16-window gate + bench match time per setting
set -e
mkdir -p gpurun_out/r04g
for g in "" "64,2" "48,2" "32,2" "32,4" "24,4"; do
  if [ -n "$g" ]; then export ZT_DF_GREAT=$g; else unset ZT_DF_GREAT; fi
  timeout -k 10 300 python tools/ratio_gate.py > gpurun_out/r04g/gate_$g.log 2>&1
  timeout -k 10 300 python bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-api > gpurun_out/r04g/bench_$g.log 2>&1
  echo "[${g:-off}] $(grep -o 'worst.*' gpurun_out/r04g/gate_$g.log) | $(grep '\[' gpurun_out/r04g/gate_$g.log | sed 's/.*\] //' | cut -c1-150) | bench $(tail -1 gpurun_out/r04g/bench_$g.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["match_kernel_ms"], d["ratio"])')"
done
