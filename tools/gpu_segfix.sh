#!/bin/bash
# Empty copy segments merged (inflate_seg.hip): segment counts, kernel stats
# A/B on the bench, inflate parity tests.
set -e
mkdir -p gpurun_out/segfix
ZT_INF_DEBUG=1 timeout -k 10 300 python3 tools/seg_probe.py > gpurun_out/segfix/probe.log 2>&1
grep "segments" gpurun_out/segfix/probe.log
bash tools/gpu_kab.sh segfix_kab ref=zlib.ts_amd/build/var_ref/libzt.so new=new 2>&1 | grep -E "==|copy_kernel|expand_kernel|tokenize"
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_inflate.py tests/test_gpu_inflate_general.py tests/test_gpu_c2.py tests/test_gpu_deflate.py tests/test_gpu_api_pipeline.py tests/test_gpu_containers.py tests/test_gpu_zip.py > gpurun_out/segfix/pytest.log 2>&1 || { tail -30 gpurun_out/segfix/pytest.log; exit 1; }
tail -2 gpurun_out/segfix/pytest.log
