#!/bin/bash
# PMC HBM traffic of the bench workload (FETCH_SIZE, read requests by size,
# WRITE_SIZE in separate passes -> profiles/pmc_traffic.json, which bench.py
# reports as roofline.traffic when its sources match the recorded digest).
#   usage: tools/gpu_checkpoint_pmc.sh TAG
set -e
TAG=${1:-ck}
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE -f csv -d $R/gpurun_out/${TAG}_pmcf -o run -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-api --no-per-generator > $R/gpurun_out/${TAG}_pmcf.log 2>&1
timeout -s KILL 180 rocprofv3 --pmc TCC_EA0_RDREQ_32B TCC_EA0_RDREQ_64B TCC_EA0_RDREQ_128B TCC_EA0_RDREQ_DRAM_32B -f csv -d $R/gpurun_out/${TAG}_pmcq -o run -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-api --no-per-generator > $R/gpurun_out/${TAG}_pmcq.log 2>&1
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE -f csv -d $R/gpurun_out/${TAG}_pmcw -o run -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-api --no-per-generator > $R/gpurun_out/${TAG}_pmcw.log 2>&1
cd $R
python3 tools/pmc_traffic.py profiles/pmc_traffic.json gpurun_out/${TAG}_pmcf gpurun_out/${TAG}_pmcq gpurun_out/${TAG}_pmcw > gpurun_out/${TAG}_pmc.txt && cp profiles/pmc_traffic.json gpurun_out/${TAG}_pmc_traffic.json
grep -E 'match_kernel|tokenize|copy_kernel|checksum' gpurun_out/${TAG}_pmc.txt || true
# the match kernel's LDS-array and VALU busy fractions (roofline.lds): an SQ pass (6 SQ counters) + the
# kernel's average duration
cd /tmp
timeout -s KILL 180 rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_WAIT_ANY -f csv -d $R/gpurun_out/${TAG}_pmcl -o run -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-api --no-per-generator > $R/gpurun_out/${TAG}_pmcl.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/${TAG}_pmcs -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-api --no-per-generator > $R/gpurun_out/${TAG}_pmcs.log 2>&1
cd $R
python3 tools/pmc_lds.py profiles/pmc_lds.json gpurun_out/${TAG}_pmcl gpurun_out/${TAG}_pmcs/run_kernel_stats.csv > gpurun_out/${TAG}_pmc_lds.txt && cp profiles/pmc_lds.json gpurun_out/${TAG}_pmc_lds.json
cat gpurun_out/${TAG}_pmc_lds.txt
