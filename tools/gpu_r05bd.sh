#!/bin/bash
# round 5: copy_kernel's descriptor chunks ahead (-DZT_CP_AHEAD 4, 8 with an
# 8 K ring; 6 at HEAD) and expand's token chunks ahead (-DZT_RS_AHEAD 4, 8
# with a 1 K ring; 6 at HEAD) after this round's kernel changes: kernel times
O=gpurun_out/r05bd; mkdir -p $O; export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp
for v in main cpa4 cpa8 rsa4 rsa8; do
  if [ $v = main ]; then unset ZT_LIB; else export ZT_LIB=$R/zlib.ts_amd/build/r05_$v/libzt.so; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/$O/prof_$v -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-api > $R/$O/bench_$v.log 2>&1 || exit 1
done
unset ZT_LIB
cd $R
for v in main cpa4 cpa8 rsa4 rsa8; do echo "$v $(python3 -c "
import csv
for r in csv.DictReader(open('$O/prof_$v/run_kernel_stats.csv')):
  n=r['Name']
  for k in ('expand_kernel','copy_kernel'):
    if k in n: print(k[:6], round(float(r['AverageNs'])/1e6,4), end=' ')
")"; done
