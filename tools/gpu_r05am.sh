#!/bin/bash
# round 5: pass 2 with the next mark word read ahead and a token's three
# stage words read as one paired read and one more (r05_p2a) -- the inflate /
# C2 suites on it, tokenize times against main (HEAD), and the SIMT
# tokenizer's cycle split (-DZT_TK_TIME builds r05_tktime = HEAD, r05_p2att)
O=gpurun_out/r05am; mkdir -p $O; export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
V=$R/zlib.ts_amd/build/r05_p2a/libzt.so
ZT_LIB=$V timeout -k 10 300 python3 -u -m pytest tests/test_gpu_inflate.py tests/test_gpu_inflate_general.py tests/test_gpu_c2.py tests/test_gpu_stream.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
cd /tmp
for v in main p2a; do
  if [ $v = main ]; then unset ZT_LIB; else export ZT_LIB=$V; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/$O/prof_$v -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-api > $R/$O/bench_$v.log 2>&1 || exit 1
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/$O/c2_$v -o run -- python3 $R/tools/c2_bench.py 3 > $R/$O/c2_$v.log 2>&1 || exit 1
done
unset ZT_LIB
cd $R
for v in main p2a; do echo "$v $(python3 -c "
import csv
for f in ('prof','c2'):
  print(f, end=': ')
  for r in csv.DictReader(open('$O/'+f+'_$v/run_kernel_stats.csv')):
    n=r['Name']
    for k in ('tokenize_kernel','expand_kernel','copy_kernel'):
      if k in n: print(k[:4], round(float(r['AverageNs'])/1e6,4), end=' ')
")"; done
for v in tktime p2att; do
  ZT_LIB=$R/zlib.ts_amd/build/r05_$v/libzt.so timeout -k 10 300 python3 tools/tk_time.py 256 wordsalad structured mixed > $O/tk_$v.log 2>&1 || exit 1
  echo "$v"; grep -v amdgpu.ids $O/tk_$v.log
done
