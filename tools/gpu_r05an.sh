#!/bin/bash
# round 5: primary decode tables of 9 and 10 bits (-DZT_PRI; 8 at HEAD):
# fewer codes take the canonical search (three dependent LDS reads, and a
# divergent branch the whole wave runs), at more LDS per tokenize unit (9: 10
# units per CU instead of 12, 10: 8) -- the inflate / C2 suites, then kernel
# times against r05_adopt (HEAD's inflate sources)
O=gpurun_out/r05an; mkdir -p $O; export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
ok=""
for v in pri9 pri10; do
  if ZT_LIB=$R/zlib.ts_amd/build/r05_$v/libzt.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_inflate.py tests/test_gpu_inflate_general.py tests/test_gpu_c2.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_$v.log 2>&1; then
    ok="$ok $v"; echo "$v $(tail -1 $O/pytest_$v.log)"
  else
    rc=$?; echo "$v FAILED rc=$rc: $(grep -m3 -E '^(FAILED|E )' $O/pytest_$v.log)"
    [ $rc -gt 1 ] && exit 1
  fi
done
cd /tmp
for v in adopt $ok; do
  ZT_LIB=$R/zlib.ts_amd/build/r05_$v/libzt.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/$O/prof_$v -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-api > $R/$O/bench_$v.log 2>&1 || exit 1
  ZT_LIB=$R/zlib.ts_amd/build/r05_$v/libzt.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/$O/c2_$v -o run -- python3 $R/tools/c2_bench.py 3 > $R/$O/c2_$v.log 2>&1 || exit 1
done
cd $R
for v in adopt $ok; do echo "$v $(python3 -c "
import csv
for f in ('prof','c2'):
  print(f, end=': ')
  for r in csv.DictReader(open('$O/'+f+'_$v/run_kernel_stats.csv')):
    n=r['Name']
    for k in ('tokenize_kernel','expand_kernel','copy_kernel'):
      if k in n: print(k[:4], round(float(r['AverageNs'])/1e6,4), end=' ')
")"; done
