#!/bin/bash
# round 5, seventh call: candidate measurement through a per-wave queue
# (ZT_DF_MQ, with u16 heads at the same 12 240 buckets: streams must equal
# main's), u16 heads alone, and the upper bound without later measurements
set -e
O=gpurun_out/r05g; mkdir -p $O; export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for L in main r05_h16e r05_mq r05_xext0 main r05_mq; do
  if [ $L = main ]; then unset ZT_LIB; else export ZT_LIB=$R/zlib.ts_amd/build/$L/libzt.so; fi
  DF_LEVELS=6,1,9 timeout -k 10 200 python3 tools/df_digest.py wordsalad structured mixed > $O/dig_$L.log 2>&1
  echo "$L $(grep L6 $O/dig_$L.log | awk '{printf "%s %s %s %s | ", $2, $3, $5, $7}')"
  echo "   $(grep -E 'L1|L9' $O/dig_$L.log | awk '{printf "%s %s %s %s | ", $1, $2, $3, $7}')"
done
unset ZT_LIB
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_classify.py > $O/pytest_classify.log 2>&1 || { tail -30 $O/pytest_classify.log; exit 1; }
tail -1 $O/pytest_classify.log
export ZT_LIB=$R/zlib.ts_amd/build/r05_mq/libzt.so
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_deflate.py tests/test_gpu_ratio.py > $O/pytest_mq.log 2>&1 || { tail -30 $O/pytest_mq.log; exit 1; }
tail -1 $O/pytest_mq.log
cd /tmp; timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/$O/prof_mq -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-api > $R/$O/bench_mq.log 2>&1; cd $R
cut -d, -f1,4 $O/prof_mq/run_kernel_stats.csv | head -6 | sed 's/(zt::[A-Za-z]*)//; s/"zt::(anonymous namespace):://; s/"//g' | tr '\n' ' '; echo
# the DP's cut lengths priced out by a saturating subtract (no compare / VCC select): identical streams expected
export ZT_LIB=$R/zlib.ts_amd/build/r05_opsat/libzt.so
DF_LEVELS=6 timeout -k 10 200 python3 tools/df_digest.py wordsalad structured mixed > $O/dig_opsat.log 2>&1
echo "opsat $(grep L6 $O/dig_opsat.log | awk '{printf "%s %s %s %s | ", $2, $3, $5, $7}')"
cd /tmp; timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/$O/prof_opsat -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-api > $R/$O/bench_opsat.log 2>&1; cd $R
unset ZT_LIB
cd /tmp; timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/$O/prof_main -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-api > $R/$O/bench_main.log 2>&1; cd $R
for t in opsat main; do echo "$t $(grep -E 'optparse|match_kernel' $O/prof_$t/run_kernel_stats.csv | cut -d, -f1,4 | sed 's/(zt::[A-Za-z]*)//; s/"zt::(anonymous namespace):://; s/"//g' | tr '\n' ' ')"; done
