#!/bin/bash
# Kernel split of the general inflate (rocprofv3 kernel trace of the timing tool).  usage: tools/gpu_genprof.sh TAG MiB
TAG=${1:-gp}; MIB=${2:-64}
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
cd /tmp
ZT_INF_DEBUG=1 timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/${TAG}_prof -o run -- python3 $R/tools/inflate_general_time.py $MIB $R/gpurun_out/${TAG}_time.json > $R/gpurun_out/${TAG}.log 2>&1 || { tail -20 $R/gpurun_out/${TAG}.log; exit 1; }
cd $R
grep -E "units, |device" gpurun_out/${TAG}.log | head -20
cut -d, -f1-4 gpurun_out/${TAG}_prof/run_kernel_stats.csv | head -24
