#!/bin/bash
# Match-kernel probes on one corpus set: hop counts (ZT_DF_COUNT variant), cycle
# split (ZT_DF_TIME variant) and LDS PMC counters of df_sweep runs.
# usage: tools/match_probe.sh TAG
set -e
TAG=${1:-mp}
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
ZT_LIB=$R/zlib.ts_amd/build/var_count/libzt.so timeout -k 10 120 python3 tools/df_count.py wordsalad xorshift32 structured > gpurun_out/$TAG/count.log 2>&1
ZT_LIB=$R/zlib.ts_amd/build/var_time/libzt.so timeout -k 10 120 python3 tools/df_time.py wordsalad xorshift32 structured > gpurun_out/$TAG/time.log 2>&1
for k in wordsalad xorshift32 structured; do
  cd /tmp && timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_ACTIVE_INST_LDS SQ_WAVES --kernel-include-regex match_kernel -d $R/gpurun_out/$TAG/pmc_$k -o run -- python3 $R/tools/df_sweep.py $k 32,128,1,128,8,16,16,1 > $R/gpurun_out/$TAG/pmc_$k.log 2>&1
  cd $R
done
cat gpurun_out/$TAG/count.log gpurun_out/$TAG/time.log
