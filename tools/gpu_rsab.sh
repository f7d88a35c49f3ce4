#!/bin/bash
# expand token ring 1024 (in-tree) vs 512 (build/exp_rs512): bench lines alternated, 10 steps each
set -e
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
for rep in 1 2; do
  for L in "" $R/zlib.ts_amd/build/exp_rs512/libzt.so; do
    ZT_LIB=$L timeout -k 10 300 python bench.py --no-cpu-baseline --no-api --steps 10 > gpurun_out/${1}_b.log 2>&1
    N=${L:+rs512}; echo "[${N:-intree}] $(tail -n 1 gpurun_out/${1}_b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print({k: d[k] for k in ["value","ms_per_step","inflate_kernel_ms","inflate_tokenize_ms"]})')"
  done
done
