#!/bin/bash
# round 5: classify_kernel's blocks contiguous per XCD (r05_clx: a block's
# history is its predecessor's bytes, read on the same L2) against main:
# digests (identical), classify times of the bench
set -e
O=gpurun_out/r05aa; mkdir -p $O; export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
V=$R/zlib.ts_amd/build/r05_clx/libzt.so
ZT_LIB=$V DF_LEVELS=6,1 timeout -k 10 200 python3 tools/df_digest.py wordsalad structured mixed > $O/dig_clx.log 2>&1
echo "clx $(grep -E 'L6|L1' $O/dig_clx.log | awk '{printf "%s %s %s %s | ", $1, $2, $3, $5}')"
cd /tmp
for v in main clx main clx; do
  L=$R/zlib.ts_amd/libzt.so; [ $v != main ] && L=$V
  ZT_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/$O/prof_$v -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-api > $R/$O/bench_$v.log 2>&1
  echo "$v $(python3 -c "
import csv
for r in csv.DictReader(open('$R/$O/prof_$v/run_kernel_stats.csv')):
  n=r['Name']
  for k in ('classify_kernel','match_kernel'):
    if k in n: print(k, round(float(r['AverageNs'])/1e6,3), end=' ')
")"
done
