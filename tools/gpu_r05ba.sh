#!/bin/bash
# round 5: find_syncs spans per workgroup around the new default 8
# (-DZT_FS_ITER 6 / 10 / 12): the inflate / stream suites on fs12, kernel
# times of all
O=gpurun_out/r05ba; mkdir -p $O; export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
ZT_LIB=$R/zlib.ts_amd/build/r05_fs12/libzt.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_inflate.py tests/test_gpu_stream.py tests/test_gpu_deflate.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
cd /tmp
for v in main fs6 fs10 fs12; do
  if [ $v = main ]; then unset ZT_LIB; else export ZT_LIB=$R/zlib.ts_amd/build/r05_$v/libzt.so; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/$O/prof_$v -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-api > $R/$O/bench_$v.log 2>&1 || exit 1
done
unset ZT_LIB
cd $R
for v in main fs6 fs10 fs12; do echo "$v $(python3 -c "
import csv
for r in csv.DictReader(open('$O/prof_$v/run_kernel_stats.csv')):
  n=r['Name']
  for k in ('find_syncs','tokenize_kernel'):
    if k in n: print(k, round(float(r['AverageNs'])/1e6,4), end=' ')
")"; done
