#!/bin/bash
# Per-generator rocprofv3 kernel stats of the deflate + inflate pipeline (256 MiB each)
#   usage: tools/gpu_kindprof.sh TAG
set -e
TAG=${1:-kp}
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for k in wordsalad xorshift32 structured; do
  cd /tmp
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/${TAG}_$k -o run -- python3 $R/tools/kind_time.py 256 $k > $R/gpurun_out/${TAG}_$k.log 2>&1
  cd $R
  cp gpurun_out/${TAG}_$k/run_kernel_stats.csv gpurun_out/${TAG}_${k}_kernel_stats.csv
  echo "== $k: $(grep ratio gpurun_out/${TAG}_$k.log)"
  python3 -c "
import csv, re
for r in csv.DictReader(open('gpurun_out/${TAG}_${k}_kernel_stats.csv')):
    n = re.split(r'[(<]', r['Name'].replace('zt::(anonymous namespace)::', ''))[0][:28]
    print(f'  {n:28s} {int(r[\"Calls\"]):4d} {float(r[\"AverageNs\"])/1e6:8.3f} ms')
"
done
