#!/bin/bash
# Inflate / deflate parity tests and a short bench line per libzt build
# (zlib.ts_amd/build/var_NAME/libzt.so; "base" = the in-tree build).
#   usage: tools/gpu_lib_bench.sh TAG "pytest -k expr" NAME...
TAG=$1; K=$2; shift 2
mkdir -p gpurun_out; R=$PWD
for nm in "$@"; do
  lib=$R/zlib.ts_amd/libzt.so; [ "$nm" = base ] || lib=$R/zlib.ts_amd/build/var_$nm/libzt.so
  echo "== $nm"
  ZT_LIB=$lib timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$K" > gpurun_out/${TAG}_${nm}_t.log 2>&1 || { tail -20 gpurun_out/${TAG}_${nm}_t.log; exit 1; }
  tail -1 gpurun_out/${TAG}_${nm}_t.log
  ZT_LIB=$lib timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-api > gpurun_out/${TAG}_${nm}_b.log 2>&1 || { tail -5 gpurun_out/${TAG}_${nm}_b.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/${TAG}_${nm}_b.log').read().strip().splitlines()[-1]); print({k: d.get(k) for k in ['value','ms_per_step','match_kernel_ms','deflate_pipeline_ms','inflate_kernel_ms','inflate_tokenize_ms','ratio']})"
done
