#!/bin/bash
# Per-kernel average times (rocprofv3 kernel stats) of the deflate pipeline per
# corpus (128 MiB, level 6) and of the 1 GiB bench.   usage: tools/kern_split.sh TAG
set -e
TAG=${1:-ks}
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
for k in wordsalad xorshift32 structured; do
  cd /tmp && timeout -k 10 120 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/$TAG/$k -o run -- python3 $R/tools/df_sweep.py $k 32,128,1,128,8,16,16,1 > $R/gpurun_out/$TAG/$k.log 2>&1
  cd $R
  grep ratio gpurun_out/$TAG/$k.log
  python3 - <<PY
import csv
rows=list(csv.DictReader(open('gpurun_out/$TAG/$k/run_kernel_stats.csv')))
print('   ' + '  '.join('%s %.2f' % (r['Name'].split('(')[0].split('::')[-1][:14], float(r['AverageNs'])/1e6) for r in rows[:9]))
PY
done
