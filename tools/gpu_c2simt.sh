#!/bin/bash
# C2 batch inflate: SIMT body decode vs one-lane decode (ZT_TOK_SIMT=0), rocprof kernel stats
set -e
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for m in 1 0; do
  cd /tmp
  ZT_TOK_SIMT=$m timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/${1}_simt$m -o run -- python3 $R/tools/c2_bench.py 3 > $R/gpurun_out/${1}_simt$m.log 2>&1
  cd $R
  echo "[simt=$m] $(tail -n 1 gpurun_out/${1}_simt$m.log)"
  python3 -c "
import csv, re
for r in csv.DictReader(open('gpurun_out/${1}_simt$m/run_kernel_stats.csv')):
    n = re.split(r'[(<]', r['Name'].replace('zt::(anonymous namespace)::', ''))[0][:28]
    if 'rocprim' in n or 'rocclr' in n or 'at::' in n: continue
    print(f'  {n:28s} {int(r[\"Calls\"]):4d} {float(r[\"AverageNs\"])/1e6:8.3f} ms')
"
done
