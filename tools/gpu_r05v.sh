#!/bin/bash
# round 5: the 4-byte-table candidates' bytes read ahead of the walks, with
# the joined extension reads (r05_q4) against main:
# digests at levels 1 / 6 / 9 (must be identical), kernel times of the bench
set -e
O=gpurun_out/r05v; mkdir -p $O; export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
V=$R/zlib.ts_amd/build/r05_q4/libzt.so
ZT_LIB=$V DF_LEVELS=6,1,9 timeout -k 10 200 python3 tools/df_digest.py wordsalad structured mixed > $O/dig_q4.log 2>&1
echo "q4 $(grep -E 'L6|L1|L9' $O/dig_q4.log | awk '{printf "%s %s %s %s | ", $1, $2, $3, $5 " " $7}')"
cd /tmp
for v in main q4 main q4; do
  L=$R/zlib.ts_amd/libzt.so; [ $v != main ] && L=$V
  ZT_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/$O/prof_$v -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-api > $R/$O/bench_$v.log 2>&1
  echo "$v $(python3 -c "
import csv
for r in csv.DictReader(open('$R/$O/prof_$v/run_kernel_stats.csv')):
  n=r['Name']
  for k in ('match_kernel',):
    if k in n: print(k, round(float(r['AverageNs'])/1e6,3), end=' ')
")"
done
