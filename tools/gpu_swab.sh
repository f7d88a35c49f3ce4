#!/bin/bash
# match_kernel_sw (sliding window) vs match_kernel (sub-chunk barrier):
# deflate tests with sw, the 16-window ratio gate for both, bench kernel stats
set -e
R=$GRAFT_REPO_ROOT
TAG=${1:-swab}
mkdir -p gpurun_out/$TAG
ZT_DF_MATCH=sw timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_deflate.py tests/test_gpu_classify.py > gpurun_out/$TAG/pytest_sw.log 2>&1 || { tail -30 gpurun_out/$TAG/pytest_sw.log; exit 1; }
tail -1 gpurun_out/$TAG/pytest_sw.log
for m in bar sw; do
  ZT_DF_MATCH=$m timeout -k 10 300 python tools/ratio_gate.py > gpurun_out/$TAG/gate_$m.log 2>&1
  echo "gate $m: $(tail -1 gpurun_out/$TAG/gate_$m.log)"
done
export TMPDIR=/tmp
for m in bar sw; do
  cd /tmp && ZT_DF_MATCH=$m timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/$TAG/$m -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-api > $R/gpurun_out/$TAG/$m.log 2>&1
  cd $R
  echo "== $m $(tail -1 gpurun_out/$TAG/$m.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ratio"], d["deflate_pipeline_ms"], d["match_kernel_ms"])')"
done
