#!/bin/bash
# round 5, eighth call: queue measurement v2 (64-bit slots with the exact
# length: no re-measure at nice_len; 128-entry ring; a pass every 8 steps),
# its counts, and the host-API inflate pieces A/B
set -e
O=gpurun_out/r05h; mkdir -p $O; export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for L in main r05_mq main r05_mq; do
  if [ $L = main ]; then unset ZT_LIB; else export ZT_LIB=$R/zlib.ts_amd/build/$L/libzt.so; fi
  DF_LEVELS=6,1,9 timeout -k 10 200 python3 tools/df_digest.py wordsalad structured mixed > $O/dig_$L.log 2>&1
  echo "$L $(grep L6 $O/dig_$L.log | awk '{printf "%s %s %s %s | ", $2, $3, $5, $7}')"
  echo "   $(grep -E 'L1|L9' $O/dig_$L.log | awk '{printf "%s %s %s %s | ", $1, $2, $3, $7}')"
done
for L in r05_cnt r05_cntmq; do
  ZT_LIB=$R/zlib.ts_amd/build/$L/libzt.so timeout -k 10 200 python3 tools/df_count.py wordsalad structured mixed > $O/cnt_$L.log 2>&1
  echo "$L"; grep -v amdgpu.ids $O/cnt_$L.log
done
unset ZT_LIB
for e in "ZT_INF_NOPIPE=1" "ZT_INF_PIECES=4" "ZT_INF_PIECES=8" "ZT_INF_PIECES=16"; do
  env $e timeout -k 10 200 python3 tools/api_inflate_time.py > $O/api_$e.log 2>&1; tail -1 $O/api_$e.log
done
