#!/bin/bash
# Round 3, box 3: bit-sliced CRC checksum kernel (tests, timing, rocprof
# kernel stats), the suites touched since r03b, and a bench line.
#   usage: tools/gpu_r03c.sh TAG
set -e
TAG=${1:-r03c}
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_checksums.py \
  tests/test_gpu_stream.py tests/test_gpu_containers.py tests/test_gpu_zip.py tests/test_gpu_batch.py \
  tests/test_gpu_deflate.py > gpurun_out/${TAG}_pytest.log 2>&1 || { tail -60 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -2 gpurun_out/${TAG}_pytest.log
timeout -k 10 120 python tools/ck_time.py > gpurun_out/${TAG}_ck.log 2>&1
cat gpurun_out/${TAG}_ck.log | grep -v amdgpu.ids
cd /tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/${TAG}_ckprof -o run -- python3 $R/tools/ck_time.py > $R/gpurun_out/${TAG}_ckprof.log 2>&1
cd $R
cp gpurun_out/${TAG}_ckprof/run_kernel_stats.csv gpurun_out/${TAG}_ck_kernel_stats.csv
cut -d, -f1-4 gpurun_out/${TAG}_ck_kernel_stats.csv | head -6
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/${TAG}_bench.log 2>&1
tail -1 gpurun_out/${TAG}_bench.log
