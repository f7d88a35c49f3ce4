#!/bin/bash
# Checksum kernel: the GPU checksum tests, the in-tree timer and rocprofv3
# kernel stats of checksum_segments (C1: 1 GiB device-resident).
#   usage: tools/gpu_ck.sh TAG
set -e
TAG=${1:-ck}
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_checksums.py \
  tests/test_gpu_containers.py > gpurun_out/${TAG}_pytest.log 2>&1 || { tail -40 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -1 gpurun_out/${TAG}_pytest.log
timeout -k 10 120 python tools/ck_time.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/${TAG}_ck.log
cd /tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/${TAG}_ckprof -o run -- python3 $R/tools/ck_time.py > $R/gpurun_out/${TAG}_ckprof.log 2>&1
cd $R
cp gpurun_out/${TAG}_ckprof/run_kernel_stats.csv gpurun_out/${TAG}_ck_kernel_stats.csv
python3 -c "
import csv
for r in csv.DictReader(open('gpurun_out/${TAG}_ck_kernel_stats.csv')):
    print(r['Name'][:60], r['Calls'], r['AverageNs'])
"
