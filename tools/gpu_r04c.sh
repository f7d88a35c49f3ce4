#!/bin/bash
# classify_kernel variant check: its tests + deflate tests, bench kernel stats
set -e
R=$GRAFT_REPO_ROOT
TAG=${1:-r04c}
mkdir -p gpurun_out/$TAG
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_classify.py tests/test_gpu_deflate.py tests/test_gpu_ratio.py tests/test_gpu_batch.py \
  > gpurun_out/$TAG/pytest.log 2>&1 || { tail -40 gpurun_out/$TAG/pytest.log; exit 1; }
tail -1 gpurun_out/$TAG/pytest.log
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/$TAG/prof -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-api > $R/gpurun_out/$TAG/prof.log 2>&1
cd $R
cp gpurun_out/$TAG/prof/run_kernel_stats.csv gpurun_out/$TAG/kernel_stats.csv
cut -d, -f1-4 gpurun_out/$TAG/kernel_stats.csv | head -14 | sed 's/(zt::[A-Za-z]*)//; s/"zt::(anonymous namespace):://'
tail -1 gpurun_out/$TAG/prof.log | cut -c1-400
