#!/bin/bash
# Tokenizer lane overlap (ZT_SP_OVERLAP bits of the previous lane's range
# decoded unmarked before a lane's own): tests on one variant, bench inflate
# split per variant, tokenizer phase cycles with and without.
set -e
TAG=${1:-r04o}
R=$GRAFT_REPO_ROOT; mkdir -p gpurun_out/$TAG; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_deflate.py tests/test_gpu_classify.py tests/test_gpu_api_pipeline.py \
  > gpurun_out/$TAG/pytest_df.log 2>&1 || { tail -30 gpurun_out/$TAG/pytest_df.log; exit 1; }
tail -1 gpurun_out/$TAG/pytest_df.log
ZT_LIB=$R/zlib.ts_amd/build/var_ov96/libzt.so timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_inflate.py tests/test_gpu_inflate_general.py tests/test_gpu_stored_runs.py tests/test_gpu_c2.py tests/test_gpu_batch.py \
  > gpurun_out/$TAG/pytest_ov96.log 2>&1 || { tail -30 gpurun_out/$TAG/pytest_ov96.log; exit 1; }
tail -1 gpurun_out/$TAG/pytest_ov96.log
for spec in ov0=zlib.ts_amd/libzt.so f32=zlib.ts_amd/build/var_f32/libzt.so ov48=zlib.ts_amd/build/var_ov48/libzt.so ov96=zlib.ts_amd/build/var_ov96/libzt.so ov160=zlib.ts_amd/build/var_ov160/libzt.so ov0b=zlib.ts_amd/libzt.so f32b=zlib.ts_amd/build/var_f32/libzt.so; do
  name=${spec%%=*}; export ZT_LIB=$R/${spec#*=}
  timeout -k 10 300 python bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-api > gpurun_out/$TAG/bench_$name.log 2>&1
  echo "[$name] $(tail -n 1 gpurun_out/$TAG/bench_$name.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print({k: d.get(k) for k in ["value","match_kernel_ms","deflate_pipeline_ms","inflate_kernel_ms","inflate_tokenize_ms"]})')"
done
for spec in ov0=zlib.ts_amd/build/var_tktime/libzt.so ov96=zlib.ts_amd/build/var_ov96tk/libzt.so; do
  name=${spec%%=*}; export ZT_LIB=$R/${spec#*=}
  timeout -k 10 300 python3 tools/tk_time.py 256 wordsalad structured mixed > gpurun_out/$TAG/tk_$name.log 2>&1
  echo "[$name]"; grep -v amdgpu.ids gpurun_out/$TAG/tk_$name.log
done
