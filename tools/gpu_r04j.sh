#!/bin/bash
# round-4 changes on the main build: tests, gate, bench, inflate host stages
set -e
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04j
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_deflate.py tests/test_gpu_classify.py tests/test_gpu_batch.py tests/test_gpu_api_pipeline.py tests/test_gpu_c3.py \
  tests/test_gpu_inflate.py tests/test_gpu_inflate_general.py tests/test_gpu_stored_runs.py tests/test_gpu_c2.py tests/test_gpu_zip.py tests/test_gpu_containers.py tests/test_gpu_stream.py \
  > gpurun_out/r04j/pytest.log 2>&1 || { tail -40 gpurun_out/r04j/pytest.log; exit 1; }
tail -1 gpurun_out/r04j/pytest.log
timeout -k 10 600 python tools/ratio_gate.py "" "28,128,1,128,8,16,16,1" "24,128,1,128,8,16,16,1" > gpurun_out/r04j/gate.log 2>&1
grep "\[" gpurun_out/r04j/gate.log
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-api > gpurun_out/r04j/bench.log 2>&1
tail -1 gpurun_out/r04j/bench.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("bench", d["value"], d["ratio"], d["deflate_pipeline_ms"], d["match_kernel_ms"], d["inflate_kernel_ms"], d.get("ratio_vs_ref"))'
ZT_INF_TIMING=1 timeout -k 10 120 python tools/inf_timing.py > gpurun_out/r04j/inf_timing.log 2>&1
tail -14 gpurun_out/r04j/inf_timing.log
export TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/r04j/prof -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-api > $R/gpurun_out/r04j/prof.log 2>&1
cd $R && cut -d, -f1-4 gpurun_out/r04j/prof/run_kernel_stats.csv | head -16 | sed 's/(zt::[A-Za-z]*)//; s/"zt::(anonymous namespace):://'
