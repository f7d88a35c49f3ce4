#!/bin/bash
# segment size sweep: headline bench per ZT_DF_RESTART (blocks of 32 KiB per independent segment)
set -o pipefail
for r in 32 16 8; do
  echo "== restart $r"
  ZT_DF_RESTART=$r timeout -k 10 200 python -u bench.py --steps 3 --warmup 1 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print({k:d[k] for k in ('value','ratio','match_kernel_ms','deflate_pipeline_ms','inflate_kernel_ms','inflate_tokenize_ms','ratio_vs_ref') if k in d})" || exit 1
done
