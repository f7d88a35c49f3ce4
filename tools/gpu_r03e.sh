#!/bin/bash
# Round 3, box 5: checksum kernel variants (occupancy / rows per segment) and
# the ratio gate of smaller hash tables (8000 / 1024 buckets) for the match
# kernel's LDS budget.
set -e
TAG=${1:-r03e}
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in "" ck_m3 ck_r32 ck_m3r32; do
  if [ -z "$v" ]; then L=""; else L=$PWD/zlib.ts_amd/build/exp_$v/libzt.so; fi
  echo "[$v] $(ZT_LIB=$L timeout -k 10 120 python tools/ck_time.py 2>&1 | grep checksums)"
done
timeout -k 10 300 python3 tools/ratio_gate.py "" > gpurun_out/${TAG}_gate_base.log 2>&1 && echo "base $(grep '^\[' gpurun_out/${TAG}_gate_base.log)"
for v in h8k h8k2; do
  ZT_LIB=$PWD/zlib.ts_amd/build/exp_$v/libzt.so timeout -k 10 300 python3 tools/ratio_gate.py "" > gpurun_out/${TAG}_gate_$v.log 2>&1
  echo "$v $(grep '^\[' gpurun_out/${TAG}_gate_$v.log)"
done
