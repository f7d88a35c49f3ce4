#!/bin/bash
# round 5, tenth call: main = alignbyte shifts unmasked (deflate digests must
# stay), expand with the token scan kept across windows and a branch-free
# descriptor, copy's step bytes by 3-input selects, and the host output pool
# (registered buffers: DMA with no staging); the full -m gpu suite on main,
# then kernel and host-API times against r05_base (HEAD's sources); the cost
# of the near probes and of the 4-byte table (time only); C4 host stage
# rates; the bench line
set -e
O=gpurun_out/r05j; mkdir -p $O; export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
BASE=$R/zlib.ts_amd/build/r05_base/libzt.so
DF_LEVELS=6,1,9 timeout -k 10 200 python3 tools/df_digest.py wordsalad structured mixed > $O/dig_main.log 2>&1
echo "main $(grep -E 'L6|L1|L9' $O/dig_main.log | awk '{printf "%s %s %s %s | ", $1, $2, $3, $5 " " $7}')"
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/$O/prof_main -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-api > $R/$O/bench_main.log 2>&1
ZT_LIB=$BASE timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/$O/prof_base -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-api > $R/$O/bench_base.log 2>&1
cd $R
for v in main base; do echo "$v $(python3 -c "
import csv,sys
for r in csv.DictReader(open('$O/prof_$v/run_kernel_stats.csv')):
  n=r['Name']
  for k in ('tokenize_kernel','expand_kernel','copy_kernel','match_kernel'):
    if k in n: print(k, round(float(r['AverageNs'])/1e6,3), end=' ')
")"; done
timeout -k 10 200 python3 tools/api_inflate_time.py > $O/api_main.log 2>&1; tail -1 $O/api_main.log
ZT_LIB=$BASE timeout -k 10 200 python3 tools/api_inflate_time.py > $O/api_base.log 2>&1; tail -1 $O/api_base.log
ZT_DF_PARAMS="20,128,1,128,8,0,16,1" DF_LEVELS=6 timeout -k 10 200 python3 tools/df_digest.py wordsalad structured mixed > $O/dig_probe0.log 2>&1
echo "probe0 $(grep L6 $O/dig_probe0.log | awk '{printf "%s %s %s | ", $2, $5, $7}')"
ZT_LIB=$R/zlib.ts_amd/build/r05_nop4/libzt.so DF_LEVELS=6 timeout -k 10 200 python3 tools/df_digest.py wordsalad structured mixed > $O/dig_nop4.log 2>&1
echo "nop4 $(grep L6 $O/dig_nop4.log | awk '{printf "%s %s %s | ", $2, $5, $7}')"
timeout -k 10 600 python3 tools/c4_host_stages.py 10000 $O/c4_host_stages.json > $O/c4_host_stages.log 2>&1; tail -5 $O/c4_host_stages.log
timeout -k 10 300 python bench.py > $O/bench.log 2>&1; tail -1 $O/bench.log
