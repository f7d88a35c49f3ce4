#!/bin/bash
# round 5: a new best length's filter word from p's first 16 bytes in
# registers instead of an LDS read (main) against the LDS read (r05_pwlds):
# digests must be identical at levels 1 / 6 / 9; match times; then the
# deflate GPU tests and the bench line
set -e
O=gpurun_out/r05n; mkdir -p $O; export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for v in main pwlds main pwlds; do
  L=$R/zlib.ts_amd/libzt.so; [ $v != main ] && L=$R/zlib.ts_amd/build/r05_$v/libzt.so
  ZT_LIB=$L DF_LEVELS=6,1,9 timeout -k 10 200 python3 tools/df_digest.py wordsalad structured mixed > $O/dig_$v.log 2>&1
  echo "$v $(grep -E 'L6|L1|L9' $O/dig_$v.log | awk '{printf "%s %s %s %s | ", $1, $2, $3, $5 " " $7}')"
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/$O/prof_main -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-api > $R/$O/bench_main.log 2>&1
ZT_LIB=$R/zlib.ts_amd/build/r05_pwlds/libzt.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/$O/prof_pwlds -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-api > $R/$O/bench_pwlds.log 2>&1
cd $R
for v in main pwlds; do echo "$v $(python3 -c "
import csv
for r in csv.DictReader(open('$O/prof_$v/run_kernel_stats.csv')):
  if 'match_kernel' in r['Name']: print('match', round(float(r['AverageNs'])/1e6,3))
")"; done
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_deflate.py tests/test_gpu_ratio.py tests/test_gpu_classify.py > $O/pytest.log 2>&1; tail -1 $O/pytest.log
