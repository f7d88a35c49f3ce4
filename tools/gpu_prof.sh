#!/bin/bash
# Quick GPU check: deflate/inflate parity tests, then rocprofv3 kernel stats of
# a short 1 GiB bench.   usage: tools/gpu_prof.sh TAG [pytest -k expr]
set -e
TAG=${1:-prof}; K=${2:-deflate}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$K" > gpurun_out/${TAG}_t.log 2>&1 || { tail -30 gpurun_out/${TAG}_t.log; exit 1; }
tail -1 gpurun_out/${TAG}_t.log
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $GRAFT_REPO_ROOT/gpurun_out/${TAG}_prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 > $GRAFT_REPO_ROOT/gpurun_out/${TAG}_bench.log 2>&1
cd $GRAFT_REPO_ROOT
grep metric gpurun_out/${TAG}_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: d[k] for k in ('value','ratio','match_kernel_ms','deflate_pipeline_ms','inflate_kernel_ms','ratio_vs_ref') if k in d})"
python3 - <<PY
import csv
rows=list(csv.DictReader(open('gpurun_out/${TAG}_prof/run_kernel_stats.csv')))
for r in rows[:12]: print('%-40s %4s %10.3f ms' % (r['Name'].replace('zt::(anonymous namespace)::','').split('(')[0][:40], r['Calls'], float(r['AverageNs'])/1e6))
PY
