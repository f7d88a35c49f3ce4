#!/bin/bash
# LDS array occupancy of the match kernel per corpus (128 MiB, level 6):
# SQ_LDS_IDX_ACTIVE (LDS-array cycles), SQ_LDS_BANK_CONFLICT (extra cycles),
# GRBM_GUI_ACTIVE (clock) -- is the chain walk bound by the LDS array?
#   usage: tools/gpu_lds_match.sh TAG
set -e
TAG=${1:-ldsm}
R=$GRAFT_REPO_ROOT; mkdir -p gpurun_out/$TAG; export TMPDIR=/tmp
for k in wordsalad xorshift32; do
  cd /tmp
  timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU GRBM_GUI_ACTIVE --kernel-include-regex match_kernel -f csv -d $R/gpurun_out/$TAG/$k -o run -- python3 $R/tools/df_sweep.py $k 32,128,1,128,8,16,16,1 > $R/gpurun_out/$TAG/$k.log 2>&1
  cd $R
  python3 - gpurun_out/$TAG/$k/run_counter_collection.csv $k <<'PY'
import csv, sys, collections
agg = collections.defaultdict(float); disp = collections.defaultdict(set)
for r in csv.DictReader(open(sys.argv[1])):
    agg[r['Counter_Name']] += float(r['Counter_Value']); disp[r['Counter_Name']].add(r['Dispatch_Id'])
v = {k: agg[k] / len(disp[k]) for k in agg}
print(sys.argv[2], " ".join(f"{k}={x:.4g}" for k, x in sorted(v.items())))
# LDS-array cycles per CU vs the kernel's cycles per XCD (GRBM_GUI_ACTIVE sums 8 XCDs)
cyc = v['GRBM_GUI_ACTIVE'] / 8
print(f"  LDS array busy per CU: {v['SQ_LDS_IDX_ACTIVE'] / 256 / cyc:.3f} of kernel cycles; bank-conflict share {v['SQ_LDS_BANK_CONFLICT'] / max(1, v['SQ_LDS_IDX_ACTIVE']):.3f}")
PY
done
