#!/bin/bash
# ratio / time frontier: next-sub-chunk heads (matches past 4 KiB sub-chunk
# ends) x chain depth x DEFLATE group (1 = 32 KiB blocks, 2 = 64 KiB)
set -e
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04i
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_deflate.py tests/test_gpu_classify.py tests/test_gpu_batch.py tests/test_gpu_api_pipeline.py tests/test_gpu_c3.py \
  tests/test_gpu_inflate.py tests/test_gpu_inflate_general.py tests/test_gpu_stored_runs.py tests/test_gpu_c2.py tests/test_gpu_zip.py tests/test_gpu_containers.py tests/test_gpu_stream.py \
  > gpurun_out/r04i/pytest.log 2>&1 || { tail -30 gpurun_out/r04i/pytest.log; exit 1; }
tail -1 gpurun_out/r04i/pytest.log
for lib in new nohead g2; do
  if [ $lib = new ]; then unset ZT_LIB; else export ZT_LIB=$R/zlib.ts_amd/build/var_$lib/libzt.so; fi
  timeout -k 10 600 python tools/ratio_gate.py "" "28,128,1,128,8,16,16,1" "24,128,1,128,8,16,16,1" "20,128,1,128,8,16,16,1" > gpurun_out/r04i/gate_$lib.log 2>&1
  echo "== $lib"; cat gpurun_out/r04i/gate_$lib.log | grep "\["
  timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-api > gpurun_out/r04i/bench_$lib.log 2>&1
  tail -1 gpurun_out/r04i/bench_$lib.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("bench", d["value"], d["ratio"], d["deflate_pipeline_ms"], d["match_kernel_ms"], d["inflate_kernel_ms"], d["ratio_vs_ref"])'
done
unset ZT_LIB
ZT_INF_TIMING=1 timeout -k 10 120 python tools/inf_timing.py > gpurun_out/r04i/inf_timing.log 2>&1
tail -14 gpurun_out/r04i/inf_timing.log
