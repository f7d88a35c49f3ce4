#!/bin/bash
# Round 4: ADVICE fixes (zip open-ended members, bounded sync-candidate token
# slots, rocPRIM sort/scan), hand-built stored-run streams, classify_kernel
# (incompressible blocks stored without a search), config C4 at its workload,
# then the bench.
set -e
mkdir -p gpurun_out/r04a
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_classify.py tests/test_gpu_stored_runs.py tests/test_gpu_deflate.py tests/test_gpu_ratio.py \
  tests/test_gpu_zip.py tests/test_gpu_inflate.py tests/test_gpu_inflate_general.py tests/test_gpu_c2.py \
  tests/test_gpu_batch.py tests/test_gpu_containers.py \
  > gpurun_out/r04a/pytest.log 2>&1 || { tail -40 gpurun_out/r04a/pytest.log; exit 1; }
tail -2 gpurun_out/r04a/pytest.log
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-api > gpurun_out/r04a/bench.log 2>&1
tail -1 gpurun_out/r04a/bench.log
ZT_C4_RECORD=gpurun_out/r04a/c4_record.json timeout -k 10 600 python -u -m pytest -x -v -s --timeout 170 --timeout-method thread \
  tests/test_gpu_c4.py > gpurun_out/r04a/c4.log 2>&1 || { tail -40 gpurun_out/r04a/c4.log; exit 1; }
grep -E "C4|passed|failed" gpurun_out/r04a/c4.log
