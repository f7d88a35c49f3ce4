#!/bin/bash
# round 5, sixth call: the 11-VALU eq_len16 as default (digests must equal
# round 4's: wordsalad 84ca8283a0431d08, structured df13e794c0378534, mixed
# 77b8e5bf657b1ed3), the branch-free measurement update, deflate tests, gate,
# bench kernel stats
set -e
O=gpurun_out/r05f; mkdir -p $O; export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for L in main r05_bf main r05_bf; do
  if [ $L = main ]; then unset ZT_LIB; else export ZT_LIB=$R/zlib.ts_amd/build/$L/libzt.so; fi
  DF_LEVELS=6 timeout -k 10 200 python3 tools/df_digest.py wordsalad structured mixed > $O/dig_$L.log 2>&1
  echo "$L $(grep L6 $O/dig_$L.log | awk '{printf "%s %s %s %s | ", $2, $3, $5, $7}')"
done
unset ZT_LIB
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_deflate.py tests/test_gpu_ratio.py tests/test_gpu_c3.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python tools/ratio_gate.py > $O/gate_main.log 2>&1; grep -o 'wordsalad [0-9.]*.*' $O/gate_main.log
cd /tmp; timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/$O/prof_main -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-api > $R/$O/bench_main.log 2>&1; cd $R
cut -d, -f1,4 $O/prof_main/run_kernel_stats.csv | head -12 | sed 's/(zt::[A-Za-z]*)//; s/"zt::(anonymous namespace):://; s/"//g' | tr '\n' ' '; echo
tail -1 $O/bench_main.log
