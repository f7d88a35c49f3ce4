#!/bin/bash
# Round 3, first box: the new / changed GPU tests (C2 at its workload, the
# logical-device batch split, data-descriptor unzip, streaming finish), the C2
# device path under rocprofv3 (kernel stats) and the host-API rate.
#   usage: tools/gpu_r03a.sh TAG
set -e
TAG=${1:-r03a}
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_c2.py \
  "tests/test_gpu_batch.py::test_alias_devices_split" tests/test_gpu_zip.py tests/test_gpu_stream.py \
  tests/test_gpu_containers.py > gpurun_out/${TAG}_pytest.log 2>&1 || { tail -40 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -2 gpurun_out/${TAG}_pytest.log
grep -h "C2:" gpurun_out/${TAG}_pytest.log || true
ZT_BATCH_TIMING=1 timeout -k 10 300 python tools/c2_bench.py 5 > gpurun_out/${TAG}_c2.json 2> gpurun_out/${TAG}_c2_stages.log
cat gpurun_out/${TAG}_c2.json
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/${TAG}_c2prof -o run -- python3 $R/tools/c2_bench.py 5 > $R/gpurun_out/${TAG}_c2prof.log 2>&1
cd $R
cp gpurun_out/${TAG}_c2prof/run_kernel_stats.csv gpurun_out/${TAG}_c2_kernel_stats.csv
cut -d, -f1-4 gpurun_out/${TAG}_c2_kernel_stats.csv | head -12
