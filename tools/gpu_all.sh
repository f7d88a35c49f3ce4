#!/bin/bash
# One GPU-box session: build check, parity tests, bench, rocprof kernel stats.
# usage: tools/gpu_all.sh TAG [bench args...]
set -e
TAG=${1:-run}; shift || true
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1 || { tail -30 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -3 gpurun_out/${TAG}_pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1
tail -1 gpurun_out/${TAG}_smoke.log
timeout -k 10 600 python bench.py "$@" > gpurun_out/${TAG}_bench.log 2>&1
tail -1 gpurun_out/${TAG}_bench.log
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d $GRAFT_REPO_ROOT/gpurun_out/${TAG}_prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/${TAG}_prof.log 2>&1
cd $GRAFT_REPO_ROOT
find gpurun_out/${TAG}_prof -name '*kernel_stats.csv' | head -1 | xargs -I{} cp {} gpurun_out/${TAG}_kernel_stats.csv
head -8 gpurun_out/${TAG}_kernel_stats.csv
