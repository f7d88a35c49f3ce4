#!/bin/bash
# round 5, fourth call: wave-level measurement passes per pair step (count
# builds), deferred measurement re-filtered at flush (2 / 3 steps), the
# 11-VALU eq_len16, and the sparse DP cut list (gate + pipeline time)
set -e
O=gpurun_out/r05d; mkdir -p $O
for L in r05_cnt r05_cntjd; do
  ZT_LIB=$PWD/zlib.ts_amd/build/$L/libzt.so timeout -k 10 200 python3 tools/df_count.py wordsalad structured mixed > $O/cnt_$L.log 2>&1
  echo "$L"; cat $O/cnt_$L.log | grep -v amdgpu.ids
done
for L in main r05_jd2f r05_jd3f r05_jd2fe r05_e2 main; do
  if [ $L = main ]; then unset ZT_LIB; else export ZT_LIB=$PWD/zlib.ts_amd/build/$L/libzt.so; fi
  DF_LEVELS=6 timeout -k 10 200 python3 tools/df_digest.py wordsalad structured mixed > $O/dig_$L.log 2>&1
  echo "$L $(grep L6 $O/dig_$L.log | awk '{printf "%s %s %s %s | ", $2, $3, $5, $7}')"
done
for L in main r05_sparse; do
  if [ $L = main ]; then unset ZT_LIB; else export ZT_LIB=$PWD/zlib.ts_amd/build/$L/libzt.so; fi
  timeout -k 10 300 python tools/ratio_gate.py > $O/gate_$L.log 2>&1
  echo "$L $(grep -o 'wordsalad [0-9.]*.*' $O/gate_$L.log)"
  cd /tmp; timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $GRAFT_REPO_ROOT/$O/prof_$L -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-api > $GRAFT_REPO_ROOT/$O/bench_$L.log 2>&1; cd $GRAFT_REPO_ROOT
  grep -E "optparse|parse_kernel|match_kernel" $O/prof_$L/run_kernel_stats.csv | cut -d, -f1,4 | sed 's/(zt::[A-Za-z]*)//; s/"zt::(anonymous namespace):://'
done
