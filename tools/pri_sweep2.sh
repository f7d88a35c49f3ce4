#!/bin/bash
# primary-table width after the canonical-limit long-code decode (libzt_p6/p8.so copied next to libzt.so)
for v in "" _p6 _p8; do
  export ZT_LIB=$GRAFT_REPO_ROOT/zlib.ts_amd/libzt$v.so
  echo "== libzt$v"
  timeout -k 10 200 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print({k:d[k] for k in ('value','inflate_kernel_ms','inflate_tokenize_ms')})" || exit 1
done
