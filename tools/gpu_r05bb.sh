#!/bin/bash
# round 5: SIMT tokenizer lane slices of 416 / 448 bits (-DZT_SP_LANE_BITS;
# 480 at HEAD) after the per-lane first pass: the inflate / C2 suites on
# sp448, tokenize times (bench, C2) of all
O=gpurun_out/r05bb; mkdir -p $O; export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
ZT_LIB=$R/zlib.ts_amd/build/r05_sp448/libzt.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_inflate.py tests/test_gpu_inflate_general.py tests/test_gpu_c2.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
cd /tmp
for v in main sp416 sp448; do
  if [ $v = main ]; then unset ZT_LIB; else export ZT_LIB=$R/zlib.ts_amd/build/r05_$v/libzt.so; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/$O/prof_$v -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-api > $R/$O/bench_$v.log 2>&1 || exit 1
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/$O/c2_$v -o run -- python3 $R/tools/c2_bench.py 3 > $R/$O/c2_$v.log 2>&1 || exit 1
done
unset ZT_LIB
cd $R
for v in main sp416 sp448; do echo "$v $(python3 -c "
import csv
for f in ('prof','c2'):
  print(f, end=': ')
  for r in csv.DictReader(open('$O/'+f+'_$v/run_kernel_stats.csv')):
    n=r['Name']
    for k in ('tokenize_kernel',):
      if k in n: print(k[:8], round(float(r['AverageNs'])/1e6,4), end=' ')
")"; done
