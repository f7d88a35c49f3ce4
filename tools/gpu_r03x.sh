#!/bin/bash
# Round 3: word-wise stored-block copy in encode, find_syncs loads in flight: deflate / inflate tests, per-generator kernel splits, bench
set -e
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=${1:-r03x}
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_deflate.py tests/test_gpu_inflate.py tests/test_gpu_batch.py tests/test_gpu_ratio.py \
  > gpurun_out/${TAG}_pytest.log 2>&1 || { tail -40 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -n 1 gpurun_out/${TAG}_pytest.log
bash tools/gpu_kindprof.sh ${TAG}k 2>&1 | grep -E "==|encode|find_syncs"
timeout -k 10 300 python bench.py --no-cpu-baseline --no-api > gpurun_out/${TAG}_bench.log 2>&1
tail -n 1 gpurun_out/${TAG}_bench.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print({k: d[k] for k in ["value","ms_per_step","match_kernel_ms","deflate_pipeline_ms","inflate_kernel_ms","ratio"]})'
ZT_LIB=$R/zlib.ts_amd/build/exp_tktime/libzt.so timeout -k 10 300 python tools/tk_time.py 256 2>&1 | grep -v amdgpu.ids | tee gpurun_out/${TAG}_tktime.log
