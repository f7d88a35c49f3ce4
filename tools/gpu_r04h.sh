#!/bin/bash
# res carries the byte; optparse reads whole lines: tests + kernel stats of variants + traffic
set -e
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04h
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_deflate.py tests/test_gpu_classify.py tests/test_gpu_ratio.py tests/test_gpu_batch.py tests/test_gpu_api_pipeline.py \
  > gpurun_out/r04h/pytest.log 2>&1 || { tail -30 gpurun_out/r04h/pytest.log; exit 1; }
tail -1 gpurun_out/r04h/pytest.log
tools/gpu_kab.sh r04h new=new pf2w1=zlib.ts_amd/build/var_pf2w1/libzt.so pf1w1=zlib.ts_amd/build/var_pf1w1/libzt.so 2>&1 | grep -E "==|match_k|optparse|parse_k|price|encode|classify|block_k"
tools/gpu_pmc.sh r04h_pmc | grep -E "optparse|parse_kernel|price|match_kernel|encode"
