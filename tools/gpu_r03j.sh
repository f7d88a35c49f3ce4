#!/bin/bash
# Round 3: stored payloads copied by stored_fill_kernel -- inflate tests, per-generator times, bench
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_inflate.py tests/test_gpu_batch.py tests/test_gpu_stream.py tests/test_gpu_c2.py \
  > gpurun_out/r03j_pytest.log 2>&1 || { tail -40 gpurun_out/r03j_pytest.log; exit 1; }
tail -n 1 gpurun_out/r03j_pytest.log
timeout -k 10 300 python tools/kind_time.py 256 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r03j_kind.log
timeout -k 10 300 python bench.py --no-cpu-baseline --no-api > gpurun_out/r03j_bench.log 2>&1
tail -n 1 gpurun_out/r03j_bench.log
