#!/bin/bash
# round 5: expand's and copy's LDS-DMA waits count the output stores issued
# after the chunk they need, so those stores stay in flight (gfx9: one
# in-order vmcnt for loads and stores).  r05_vmw against main: the inflate
# parity suites on r05_vmw, then kernel times of the bench
set -e
O=gpurun_out/r05s; mkdir -p $O; export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
V=$R/zlib.ts_amd/build/r05_vmw/libzt.so
ZT_LIB=$V timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_inflate.py tests/test_gpu_inflate_general.py tests/test_gpu_stored_runs.py tests/test_gpu_c2.py tests/test_gpu_stream.py tests/test_gpu_api_pipeline.py > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
cd /tmp
for v in main vmw main vmw; do
  L=$R/zlib.ts_amd/libzt.so; [ $v != main ] && L=$V
  ZT_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/$O/prof_$v -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-api > $R/$O/bench_$v.log 2>&1
  echo "$v $(python3 -c "
import csv
for r in csv.DictReader(open('$R/$O/prof_$v/run_kernel_stats.csv')):
  n=r['Name']
  for k in ('tokenize_kernel','expand_kernel','copy_kernel'):
    if k in n: print(k, round(float(r['AverageNs'])/1e6,3), end=' ')
")"
done
