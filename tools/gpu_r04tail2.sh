#!/bin/bash
# tail workgroups with larger main ones (ZT_DF_SUPER x ZT_DF_TAILR, ZT_DF_TAILK 1)
set -e
mkdir -p gpurun_out/r04tail2
for sr in 4:1 8:1 8:2 8:3 4:1 8:2; do
  k=${sr%%:*}; r=${sr#*:}
  ZT_DF_SUPER=$k ZT_DF_TAILK=1 ZT_DF_TAILR=$r timeout -k 10 300 python bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-api > gpurun_out/r04tail2/bench_$k$r.log 2>&1
  echo "[super $k tail rounds $r] $(tail -1 gpurun_out/r04tail2/bench_$k$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["deflate_pipeline_ms"], d["match_kernel_ms"], d["ratio"])')"
done
