#!/bin/bash
# Counters of the checksum kernel on 1 GiB (tools/ck_time.py), one pass per group.
set -e
TAG=${1:-ck}; R=$PWD; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 120 python3 tools/ck_time.py
cd /tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS -f csv -d $R/gpurun_out/${TAG}_sq -o run -- python3 $R/tools/ck_time.py > /dev/null 2>&1
timeout -s KILL 90 rocprofv3 --pmc TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TA_BUSY_avr TCC_HIT_sum -f csv -d $R/gpurun_out/${TAG}_tcp -o run -- python3 $R/tools/ck_time.py > /dev/null 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES GRBM_GUI_ACTIVE TCC_MISS_sum -f csv -d $R/gpurun_out/${TAG}_lds -o run -- python3 $R/tools/ck_time.py > /dev/null 2>&1
cd $R
for d in sq tcp lds; do python3 - gpurun_out/${TAG}_$d/run_counter_collection.csv <<'PY'
import csv, sys, collections
agg = collections.defaultdict(float); disp = collections.defaultdict(set)
for r in csv.DictReader(open(sys.argv[1])):
    if 'checksum_segments' not in r['Kernel_Name']: continue
    agg[r['Counter_Name']] += float(r['Counter_Value']); disp[r['Counter_Name']].add(r['Dispatch_Id'])
for k, v in agg.items(): print(f"{k:32s} {v/len(disp[k]):14.4g} per dispatch")
PY
done
