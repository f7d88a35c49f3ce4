#!/bin/bash
# C3 checks: full-size 8 GiB round trip test, sharded layout, bench launcher
# modes, then the C3 bench line at N=1.   usage: tools/gpu_c3.sh TAG
set -e
TAG=${1:-c3}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_c3.py -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_t.log 2>&1 || { tail -40 gpurun_out/${TAG}_t.log; exit 1; }
tail -3 gpurun_out/${TAG}_t.log
timeout -k 10 300 python bench.py --mode c3 --steps 3 --warmup 1 > gpurun_out/${TAG}_bench_c3.log 2>&1
tail -1 gpurun_out/${TAG}_bench_c3.log
timeout -k 10 300 python bench.py > gpurun_out/${TAG}_bench.log 2>&1
tail -1 gpurun_out/${TAG}_bench.log
