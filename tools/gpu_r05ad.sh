#!/bin/bash
# round 5: the link waves at a higher issue priority (s_setprio 1 / 3 while
# linking; round 2 measured it slower on a different kernel) against main:
# match times of the bench (the link is on every sub-chunk's critical path)
set -e
O=gpurun_out/r05ad; mkdir -p $O; export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp
for v in main prio1 prio3 main prio1 prio3; do
  L=$R/zlib.ts_amd/libzt.so; [ $v != main ] && L=$R/zlib.ts_amd/build/r05_$v/libzt.so
  ZT_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/$O/prof_$v -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-api > $R/$O/bench_$v.log 2>&1
  echo "$v $(python3 -c "
import csv
for r in csv.DictReader(open('$R/$O/prof_$v/run_kernel_stats.csv')):
  if 'match_kernel' in r['Name']: print('match', round(float(r['AverageNs'])/1e6,3))
")"
done
