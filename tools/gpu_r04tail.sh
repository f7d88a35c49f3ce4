#!/bin/bash
# smaller match workgroups for the last round (ZT_DF_TAILK blocks each over
# ZT_DF_TAILR rounds of num_cu workgroups): streams identical, bench per setting
set -e
mkdir -p gpurun_out/r04tail
ZT_DF_TAILK=0 timeout -k 10 300 python tools/df_digest.py mixed > gpurun_out/r04tail/digest_0.log 2>&1
timeout -k 10 300 python tools/df_digest.py mixed > gpurun_out/r04tail/digest_1.log 2>&1
diff <(awk '{print $1,$2,$3}' gpurun_out/r04tail/digest_0.log) <(awk '{print $1,$2,$3}' gpurun_out/r04tail/digest_1.log) && echo "digests identical"
for kr in 0:1 1:1 2:1 1:2 2:2 0:1 1:1; do
  k=${kr%%:*}; r=${kr#*:}
  ZT_DF_TAILK=$k ZT_DF_TAILR=$r timeout -k 10 300 python bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-api > gpurun_out/r04tail/bench_$k$r.log 2>&1
  echo "[tailk $k rounds $r] $(tail -1 gpurun_out/r04tail/bench_$k$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["deflate_pipeline_ms"], d["match_kernel_ms"], d["ratio"])')"
done
