#!/bin/bash
# sequential carried walks (var_seq): level-6 frontier (chain, good) on the gate + bench
set -e
R=$GRAFT_REPO_ROOT; mkdir -p gpurun_out/r04s2
export ZT_LIB=$R/zlib.ts_amd/build/var_seq/libzt.so
for ps in "28,128,1,128,8,16,24,1" "28,128,1,128,8,16,32,1" "28,128,1,128,8,16,258,1" "32,128,1,128,8,16,24,1" "24,128,1,128,8,16,32,1" "32,128,1,128,8,16,258,1"; do
  timeout -k 10 300 python tools/ratio_gate.py "$ps" > gpurun_out/r04s2/gate_$ps.log 2>&1
  ZT_DF_PARAMS=$ps timeout -k 10 300 python bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-api > gpurun_out/r04s2/bench_$ps.log 2>&1
  echo "$ps | $(grep '\[' gpurun_out/r04s2/gate_$ps.log | sed 's/.*\] //' | cut -c1-170) | bench $(tail -1 gpurun_out/r04s2/bench_$ps.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["match_kernel_ms"], d["ratio"])')"
done
