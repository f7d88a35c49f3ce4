#!/bin/bash
# blocks per match workgroup (ZT_DF_SUPER) on the headline bench
for k in 4 2 1 4; do
  echo "== super $k"
  ZT_DF_SUPER=$k timeout -k 10 200 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print({k:d[k] for k in ('value','ratio','match_kernel_ms','deflate_pipeline_ms','inflate_kernel_ms')})" || exit 1
done
