#!/bin/bash
# Stored runs as run tokens expanded from the input (no stored_fill pass):
# inflate parity tests, then kernel stats A/B on the bench and per generator.
set -e
mkdir -p gpurun_out/runtok
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_inflate.py tests/test_gpu_inflate_general.py tests/test_gpu_c2.py tests/test_gpu_stream.py tests/test_gpu_containers.py tests/test_gpu_zip.py tests/test_gpu_batch.py tests/test_gpu_api_pipeline.py > gpurun_out/runtok/pytest.log 2>&1 || { tail -40 gpurun_out/runtok/pytest.log; exit 1; }
tail -2 gpurun_out/runtok/pytest.log
bash tools/gpu_kab.sh runtok_kab ref=zlib.ts_amd/build/var_ref/libzt.so new=new 2>&1 | grep -E "==|copy_kernel|expand_kernel|tokenize|stored_fill"
ZT_LIB=$PWD/zlib.ts_amd/build/var_ref/libzt.so timeout -k 10 300 python3 -u tools/kind_time.py > gpurun_out/runtok/kind_ref.log 2>&1
timeout -k 10 300 python3 -u tools/kind_time.py > gpurun_out/runtok/kind_new.log 2>&1
cat gpurun_out/runtok/kind_ref.log gpurun_out/runtok/kind_new.log | grep ratio
