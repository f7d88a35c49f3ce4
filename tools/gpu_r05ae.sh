#!/bin/bash
# round 5: copy_kernel with its per-step offsets in 32 bits (segments below
# 2^31 bytes) -- the inflate suites on that build, then kernel times of main
# (HEAD) and the variant under rocprofv3
set -e
O=gpurun_out/r05ae; mkdir -p $O; export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
VAR=$R/zlib.ts_amd/build/r05_cp32/libzt.so
ZT_LIB=$VAR timeout -k 10 600 python3 -u -m pytest tests/test_gpu_inflate.py tests/test_gpu_inflate_general.py tests/test_gpu_stored_runs.py tests/test_gpu_stream.py tests/test_gpu_c3.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/$O/prof_main -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-api > $R/$O/bench_main.log 2>&1
ZT_LIB=$VAR timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/$O/prof_var -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-api > $R/$O/bench_var.log 2>&1
cd $R
for v in main var; do echo "$v $(python3 -c "
import csv,sys
for r in csv.DictReader(open('$O/prof_$v/run_kernel_stats.csv')):
  n=r['Name']
  for k in ('tokenize_kernel','expand_kernel','copy_kernel','find_syncs','chain'):
    if k in n: print(k, round(float(r['AverageNs'])/1e6,4), end=' ')
")"; done
