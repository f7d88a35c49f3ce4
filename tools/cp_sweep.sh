#!/bin/bash
# copy_kernel descriptor prefetch depth (variant builds): inflate tests + bench per variant
for v in "" var_cp20/ var_cp28/; do
  if [ -n "$v" ]; then export ZT_LIB=$GRAFT_REPO_ROOT/zlib.ts_amd/build/${v}libzt.so; fi
  echo "== ${v:-default}"
  timeout -k 10 200 python -u -m pytest tests -m gpu -x -q -k "inflate or two_phase or roundtrip" --timeout 120 --timeout-method thread 2>&1 | tail -1 || exit 1
  timeout -k 10 200 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print({k:d[k] for k in ('value','inflate_kernel_ms','inflate_tokenize_ms')})" || exit 1
done
