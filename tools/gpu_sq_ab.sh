#!/bin/bash
# SQ counters of the match kernel for two libzt builds (ref vs in-tree) on one corpus.
#   usage: tools/gpu_sq_ab.sh TAG KIND
set -e
TAG=${1:-sq}; KIND=${2:-wordsalad}
R=$PWD; mkdir -p gpurun_out; export TMPDIR=/tmp
C="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS"
for v in ref new; do
  if [ $v = ref ]; then export ZT_LIB=$R/zlib.ts_amd/build/ref/libzt.so; else unset ZT_LIB; fi
  cd /tmp
  timeout -s KILL 120 rocprofv3 --pmc $C -f csv -d $R/gpurun_out/${TAG}_$v -o run -- python3 $R/tools/df_digest.py $KIND > $R/gpurun_out/${TAG}_$v.log 2>&1
  cd $R
  python3 tools/sq_summ.py gpurun_out/${TAG}_$v/run_counter_collection.csv | grep match_kernel | sed "s/^/$v /"
done
