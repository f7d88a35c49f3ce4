#!/bin/bash
# inflate chain on the device (in-tree) vs the host walk (ZT_INF_HOST_CHAIN=1):
# tests, bench inflate time (interleaved), host stage times, kernel stats
set -e
TAG=${1:-r04dc}
R=$GRAFT_REPO_ROOT; mkdir -p gpurun_out/$TAG; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_deflate.py tests/test_gpu_inflate.py tests/test_gpu_inflate_general.py tests/test_gpu_stored_runs.py tests/test_gpu_c2.py tests/test_gpu_batch.py tests/test_gpu_stream.py tests/test_gpu_c3.py tests/test_gpu_api_pipeline.py \
  > gpurun_out/$TAG/pytest.log 2>&1 || { tail -30 gpurun_out/$TAG/pytest.log; exit 1; }
tail -1 gpurun_out/$TAG/pytest.log
for mode in dev host dev2 host2; do
  if [ "${mode#host}" != "$mode" ]; then export ZT_INF_HOST_CHAIN=1; else unset ZT_INF_HOST_CHAIN; fi
  timeout -k 10 300 python bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-api > gpurun_out/$TAG/bench_$mode.log 2>&1
  echo "[$mode] $(tail -n 1 gpurun_out/$TAG/bench_$mode.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print({k: d.get(k) for k in ["value","deflate_pipeline_ms","inflate_kernel_ms","inflate_tokenize_ms"]})')"
done
unset ZT_INF_HOST_CHAIN
ZT_INF_TIMING=1 timeout -k 10 120 python tools/inf_timing.py > gpurun_out/$TAG/inf_timing.log 2>&1
tail -14 gpurun_out/$TAG/inf_timing.log
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/$TAG/prof -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-api > $R/gpurun_out/$TAG/prof.log 2>&1
cd $R && cut -d, -f1-4 gpurun_out/$TAG/prof/run_kernel_stats.csv | head -18 | sed 's/(zt::[A-Za-z]*)//; s/"zt::(anonymous namespace):://'
