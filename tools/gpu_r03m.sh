#!/bin/bash
# Round 3: copy kernels with 1 KiB descriptor DMAs + unrolled flush: inflate tests, phase cycles, bench
set -e
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=${1:-r03m}
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_inflate.py tests/test_gpu_inflate_general.py tests/test_gpu_batch.py tests/test_gpu_c2.py \
  > gpurun_out/${TAG}_pytest.log 2>&1 || { tail -40 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -n 1 gpurun_out/${TAG}_pytest.log
ZT_LIB=$R/zlib.ts_amd/build/exp_cptime/libzt.so timeout -k 10 200 python tools/cp_time.py 1024 mixed 2>&1 | grep -v amdgpu.ids | tee gpurun_out/${TAG}_cptime.log
timeout -k 10 300 python bench.py --no-cpu-baseline --no-api > gpurun_out/${TAG}_bench.log 2>&1
tail -n 1 gpurun_out/${TAG}_bench.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print({k: d[k] for k in ["value","ms_per_step","match_kernel_ms","deflate_pipeline_ms","inflate_kernel_ms","inflate_tokenize_ms"]})'
