#!/bin/bash
# round 5: the cost of codes longer than the 8-bit primary table at equal
# occupancy -- r05_pri10 (10-bit tables, 8 tokenize units per CU) against
# r05_pad6k (8-bit tables with the same LDS, -DZT_TOK_LDS_PAD=6144): kernel
# times (bench, C2) and the cycle split per corpus (-DZT_TK_TIME builds)
O=gpurun_out/r05ao; mkdir -p $O; export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp
for v in pad6k pri10; do
  export ZT_LIB=$R/zlib.ts_amd/build/r05_$v/libzt.so
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/$O/prof_$v -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-api > $R/$O/bench_$v.log 2>&1 || exit 1
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/$O/c2_$v -o run -- python3 $R/tools/c2_bench.py 3 > $R/$O/c2_$v.log 2>&1 || exit 1
done
unset ZT_LIB
cd $R
for v in pad6k pri10; do echo "$v $(python3 -c "
import csv
for f in ('prof','c2'):
  print(f, end=': ')
  for r in csv.DictReader(open('$O/'+f+'_$v/run_kernel_stats.csv')):
    n=r['Name']
    for k in ('tokenize_kernel','expand_kernel','copy_kernel'):
      if k in n: print(k[:4], round(float(r['AverageNs'])/1e6,4), end=' ')
")"; done
for v in pad6ktt pri10tt; do
  ZT_LIB=$R/zlib.ts_amd/build/r05_$v/libzt.so timeout -k 10 300 python3 tools/tk_time.py 256 wordsalad structured mixed > $O/tk_$v.log 2>&1 || exit 1
  echo "$v"; grep -v amdgpu.ids $O/tk_$v.log
done
