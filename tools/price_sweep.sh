#!/bin/bash
# price statistics sample (1/ZT_PRICE_SAMPLE of each block) on the headline bench
for v in "" var_ps2/ var_ps1/; do
  if [ -n "$v" ]; then export ZT_LIB=$GRAFT_REPO_ROOT/zlib.ts_amd/build/${v}libzt.so; fi
  echo "== ${v:-default}"
  timeout -k 10 200 python -u bench.py --steps 3 --warmup 1 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print({k:d[k] for k in ('value','ratio','deflate_pipeline_ms','ratio_vs_ref')})" || exit 1
done
