#!/bin/bash
# round 5: the first pass and the repairs decode one code per lane per
# iteration (a token's length and distance codes in separate iterations, the
# table picked per lane) -- the inflate / C2 / batch suites on that build,
# then tokenize times (bench and C2 batch) against r05_lbpf
set -e
O=gpurun_out/r05ag; mkdir -p $O; export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
VAR=$R/zlib.ts_amd/build/r05_lcode/libzt.so
BASE=$R/zlib.ts_amd/build/r05_lbpf/libzt.so
ZT_LIB=$VAR timeout -k 10 600 python3 -u -m pytest tests/test_gpu_inflate.py tests/test_gpu_inflate_general.py tests/test_gpu_stored_runs.py tests/test_gpu_stream.py tests/test_gpu_c2.py tests/test_gpu_c3.py tests/test_gpu_batch.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
cd /tmp
for v in base var; do
  L=$BASE; [ $v = var ] && L=$VAR
  ZT_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/$O/prof_$v -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-api > $R/$O/bench_$v.log 2>&1
  ZT_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/$O/c2_$v -o run -- python3 $R/tools/c2_bench.py 3 > $R/$O/c2_$v.log 2>&1
done
cd $R
for v in base var; do echo "$v $(python3 -c "
import csv,sys
for f in ('prof','c2'):
  print(f, end=': ')
  for r in csv.DictReader(open('$O/'+f+'_$v/run_kernel_stats.csv')):
    n=r['Name']
    for k in ('tokenize_kernel','expand_kernel','copy_kernel','batch'):
      if k in n: print(n.split('(')[0][-30:], round(float(r['AverageNs'])/1e6,4), r['Calls'], end=' ')
")"; done
