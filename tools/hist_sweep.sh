#!/bin/bash
# history bytes per match super-chunk (ZT_DF_HIST KiB) x super-chunk size on the headline bench
for h in 28 20 16; do for k in 4 8; do
  echo "== hist $h KiB super $k"
  ZT_DF_HIST=$h ZT_DF_SUPER=$k timeout -k 10 200 python -u bench.py --steps 3 --warmup 1 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print({k:d[k] for k in ('value','ratio','match_kernel_ms','ratio_vs_ref')})" || exit 1
done; done
