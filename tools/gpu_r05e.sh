#!/bin/bash
# round 5, fifth call: 11-VALU eq_len16 (identical streams), the sparse DP
# cut list and u16 heads at chain 19 / 20: gate + kernel stats of the bench
set -e
O=gpurun_out/r05e; mkdir -p $O; export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for L in main r05_e2 main r05_e2; do
  if [ $L = main ]; then unset ZT_LIB; else export ZT_LIB=$R/zlib.ts_amd/build/$L/libzt.so; fi
  DF_LEVELS=6 timeout -k 10 200 python3 tools/df_digest.py wordsalad structured mixed > $O/dig_$L.log 2>&1
  echo "$L $(grep L6 $O/dig_$L.log | awk '{printf "%s %s %s %s | ", $2, $3, $5, $7}')"
done
run() {  # tag lib params
  if [ $2 = main ]; then unset ZT_LIB; else export ZT_LIB=$R/zlib.ts_amd/build/$2/libzt.so; fi
  if [ -n "$3" ]; then export ZT_DF_PARAMS=$3; else unset ZT_DF_PARAMS; fi
  timeout -k 10 300 python tools/ratio_gate.py > $O/gate_$1.log 2>&1
  echo "$1 $(grep -o 'wordsalad [0-9.]*.*' $O/gate_$1.log)"
  cd /tmp; timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/$O/prof_$1 -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-api > $R/$O/bench_$1.log 2>&1; cd $R
  echo "   $(grep -E 'match_kernel|optparse|parse_kernel' $O/prof_$1/run_kernel_stats.csv | cut -d, -f1,4 | sed 's/(zt::[A-Za-z]*)//; s/"zt::(anonymous namespace):://; s/"//g' | tr '\n' ' ')"
}
run main main ""
run sparse r05_sparse ""
run h16 r05_h16 ""
run h16c19 r05_h16 "19,128,1,128,8,16,16,1"
run sparse_c22 r05_sparse "22,128,1,128,8,16,16,1"
