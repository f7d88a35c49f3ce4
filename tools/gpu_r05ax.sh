#!/bin/bash
# round 5: the DP pairs masked independently and reduced by a min3 tree
# (r05_optree, -DZT_OP_TREE): digests at levels 6 / 1 / 9 against main,
# then the deflate kernel times of both
O=gpurun_out/r05ax; mkdir -p $O; export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
V=$R/zlib.ts_amd/build/r05_optree/libzt.so
for v in main optree; do
  if [ $v = main ]; then unset ZT_LIB; else export ZT_LIB=$V; fi
  DF_LEVELS=6,1,9 timeout -k 10 300 python3 tools/df_digest.py wordsalad structured mixed > $O/dig_$v.log 2>&1 || exit 1
  echo "$v $(grep -E 'L6|L1|L9' $O/dig_$v.log | awk '{printf "%s %s %s | ", $1, $2, $3}')"
done
cd /tmp
for v in main optree; do
  if [ $v = main ]; then unset ZT_LIB; else export ZT_LIB=$V; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/$O/prof_$v -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-api > $R/$O/bench_$v.log 2>&1 || exit 1
done
unset ZT_LIB
cd $R
for v in main optree; do echo "$v $(python3 -c "
import csv
for r in csv.DictReader(open('$O/prof_$v/run_kernel_stats.csv')):
  n=r['Name']
  for k in ('optparse_kernel','match_kernel','parse_kernel'):
    if k in n: print(k[:8], round(float(r['AverageNs'])/1e6,4), end=' ')
")"; done
