#!/bin/bash
# calibrated HBM traffic per kernel of the bench (tools/pmc_traffic.py)
set -e
R=$GRAFT_REPO_ROOT
TAG=${1:-pmc}
mkdir -p gpurun_out/$TAG
cd /tmp
B="python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-api"
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE -f csv -d $R/gpurun_out/$TAG/f -o run -- $B > $R/gpurun_out/$TAG/f.log 2>&1
timeout -s KILL 180 rocprofv3 --pmc TCC_EA0_RDREQ_32B TCC_EA0_RDREQ_64B TCC_EA0_RDREQ_128B TCC_EA0_RDREQ_DRAM_32B -f csv -d $R/gpurun_out/$TAG/q -o run -- $B > $R/gpurun_out/$TAG/q.log 2>&1
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE -f csv -d $R/gpurun_out/$TAG/w -o run -- $B > $R/gpurun_out/$TAG/w.log 2>&1
cd $R
python3 tools/pmc_traffic.py gpurun_out/$TAG/pmc_traffic.json gpurun_out/$TAG/f gpurun_out/$TAG/q gpurun_out/$TAG/w | tee gpurun_out/$TAG/pmc.txt
