#!/bin/bash
# primary-table width sweep: headline bench (tokenize ms) + C2 per-corpus latency per library variant
set -o pipefail
for v in "" _pri8 _pri9; do
  export ZT_LIB=$GRAFT_REPO_ROOT/zlib.ts_amd/libzt$v.so
  echo "== libzt$v"
  timeout -k 10 200 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print({k:d[k] for k in ('value','inflate_kernel_ms','inflate_tokenize_ms')})" || exit 1
  timeout -k 10 120 python -u tools/c2_kind.py 2>/dev/null || exit 1
done
