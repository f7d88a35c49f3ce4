#!/bin/bash
# round 5: the first pass keeps its tokens (a scratch slot per wave) and pass
# 2 copies them, decoding only tokens a repair re-marked (r05_spec) -- the
# inflate / stream / pipeline / thread / C2 / C3 suites on it, then kernel
# times against main (bench, C2)
O=gpurun_out/r05at; mkdir -p $O; export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
V=$R/zlib.ts_amd/build/r05_spec/libzt.so
ZT_LIB=$V timeout -k 10 900 python3 -u -m pytest tests/test_gpu_inflate.py tests/test_gpu_inflate_general.py tests/test_gpu_stream.py tests/test_gpu_stored_runs.py tests/test_gpu_api_pipeline.py tests/test_gpu_threads.py tests/test_gpu_c2.py tests/test_gpu_c3.py tests/test_gpu_deflate.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
cd /tmp
for v in main spec; do
  if [ $v = main ]; then unset ZT_LIB; else export ZT_LIB=$V; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/$O/prof_$v -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-api > $R/$O/bench_$v.log 2>&1 || exit 1
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/$O/c2_$v -o run -- python3 $R/tools/c2_bench.py 3 > $R/$O/c2_$v.log 2>&1 || exit 1
done
unset ZT_LIB
cd $R
for v in main spec; do echo "$v $(python3 -c "
import csv
for f in ('prof','c2'):
  print(f, end=': ')
  for r in csv.DictReader(open('$O/'+f+'_$v/run_kernel_stats.csv')):
    n=r['Name']
    for k in ('tokenize_kernel','expand_kernel','copy_kernel'):
      if k in n: print(k[:6], round(float(r['AverageNs'])/1e6,4), end=' ')
")"; done
