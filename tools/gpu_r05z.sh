#!/bin/bash
# round 5: restart points every 512 KiB instead of 1 MiB (ZT_DF_RESTART=16
# blocks): twice the copy segments (copy_kernel runs one wave per segment,
# one per SIMD at 1 MiB) against the ratio the extra history-free starts
# cost -- the 16-window gate and the bench's kernel times
set -e
O=gpurun_out/r05z; mkdir -p $O; export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
ZT_DF_RESTART=16 timeout -k 10 300 python3 tools/ratio_gate.py > $O/gate_r16.log 2>&1; tail -1 $O/gate_r16.log
cd /tmp
for v in 32 16; do
  ZT_DF_RESTART=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/$O/prof_$v -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-api > $R/$O/bench_$v.log 2>&1
  echo "restart $v: $(tail -1 $R/$O/bench_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ratio'], d['deflate_pipeline_ms'], d['inflate_kernel_ms'])") $(python3 -c "
import csv
for r in csv.DictReader(open('$R/$O/prof_$v/run_kernel_stats.csv')):
  n=r['Name']
  for k in ('match_kernel','tokenize_kernel','expand_kernel','copy_kernel'):
    if k in n: print(k, round(float(r['AverageNs'])/1e6,3), end=' ')
")"
done
