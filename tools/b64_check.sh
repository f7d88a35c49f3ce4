#!/bin/bash
# 64 KiB deflate blocks (variant build): GPU tests, then the bench at 1 MiB and 512 KiB segments
export ZT_LIB=$GRAFT_REPO_ROOT/zlib.ts_amd/build/var_b64/libzt.so
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/b64_t.log 2>&1; tail -3 gpurun_out/b64_t.log
for r in 16 8; do
  echo "== restart $r blocks"
  ZT_DF_RESTART=$r timeout -k 10 200 python -u bench.py --steps 3 --warmup 1 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print({k:d[k] for k in ('value','ratio','match_kernel_ms','deflate_pipeline_ms','inflate_kernel_ms','inflate_tokenize_ms','ratio_vs_ref')})" || exit 1
done
