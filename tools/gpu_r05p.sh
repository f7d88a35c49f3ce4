#!/bin/bash
# round 5: the hop's filter-word reads issued before its link reads (r05_ford;
# LDS reads complete in order and the checks need the filter words first)
# against main: digests at levels 1 / 6 / 9 (must be identical), match times
set -e
O=gpurun_out/r05p; mkdir -p $O; export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for v in main ford main ford; do
  L=$R/zlib.ts_amd/libzt.so; [ $v != main ] && L=$R/zlib.ts_amd/build/r05_$v/libzt.so
  ZT_LIB=$L DF_LEVELS=6,1,9 timeout -k 10 200 python3 tools/df_digest.py wordsalad structured mixed > $O/dig_$v.log 2>&1
  echo "$v $(grep -E 'L6|L1|L9' $O/dig_$v.log | awk '{printf "%s %s %s %s | ", $1, $2, $3, $5 " " $7}')"
done
cd /tmp
for v in main ford; do
  L=$R/zlib.ts_amd/libzt.so; [ $v != main ] && L=$R/zlib.ts_amd/build/r05_$v/libzt.so
  ZT_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/$O/prof_$v -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-api > $R/$O/bench_$v.log 2>&1
  echo "$v $(python3 -c "
import csv
for r in csv.DictReader(open('$R/$O/prof_$v/run_kernel_stats.csv')):
  if 'match_kernel' in r['Name']: print('match', round(float(r['AverageNs'])/1e6,3))
")"
done
