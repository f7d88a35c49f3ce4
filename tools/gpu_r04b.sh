#!/bin/bash
# rocprof kernel stats of the bench and of config C4 (tools/c4_batch.py)
set -e
R=$GRAFT_REPO_ROOT
TAG=${1:-r04b}
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/$TAG/prof -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-api > $R/gpurun_out/$TAG/prof.log 2>&1
cd $R
cp gpurun_out/$TAG/prof/run_kernel_stats.csv gpurun_out/$TAG/kernel_stats.csv
cut -d, -f1-4 gpurun_out/$TAG/kernel_stats.csv | head -16
timeout -k 10 400 python3 tools/c4_batch.py 10000 gpurun_out/$TAG/c4_batch.json > gpurun_out/$TAG/c4_batch.log 2>&1
tail -3 gpurun_out/$TAG/c4_batch.log
