#!/bin/bash
# round 5: copy steps of 2 KiB with 4 descriptor chunks ahead (the 16 KiB
# descriptor ring of r05l's cp2k left 3 copy workgroups per CU), 4 KiB steps,
# and a 256-token expand ring (expand's LDS grows with the copy step): kernel
# times of the bench (rocprof) against main and r05l's cp2k
set -e
O=gpurun_out/r05m; mkdir -p $O; export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp
for v in main cp2k cp2ka4 cp2ka4t256 cp4k t256; do
  L=$R/zlib.ts_amd/libzt.so; [ $v != main ] && L=$R/zlib.ts_amd/build/r05_$v/libzt.so
  ZT_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/$O/prof_$v -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-api > $R/$O/bench_$v.log 2>&1
  echo "$v $(python3 -c "
import csv
for r in csv.DictReader(open('$R/$O/prof_$v/run_kernel_stats.csv')):
  n=r['Name']
  for k in ('tokenize_kernel','expand_kernel','copy_kernel'):
    if k in n: print(k, round(float(r['AverageNs'])/1e6,3), end=' ')
")"
done
