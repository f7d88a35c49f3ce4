#!/bin/bash
# A/B of a deflate variant (build/exp_NAME) against the in-tree library:
# deflate tests on the variant, ratio gate, per-generator times and bench for both.
#   usage: tools/gpu_varab.sh TAG NAME
set -e
TAG=$1; V=$2
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
VL=$R/zlib.ts_amd/build/exp_$V/libzt.so
ZT_LIB=$VL timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_deflate.py \
  > gpurun_out/${TAG}_pytest.log 2>&1 || { tail -30 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -n 1 gpurun_out/${TAG}_pytest.log
for L in "" $VL; do
  N=${L:+$V}; N=${N:-in-tree}
  ZT_LIB=$L timeout -k 10 300 python3 tools/ratio_gate.py "" > gpurun_out/${TAG}_gate_$N.log 2>&1
  echo "[$N] $(grep '^\[' gpurun_out/${TAG}_gate_$N.log)"
  ZT_LIB=$L timeout -k 10 300 python tools/kind_time.py 256 2>&1 | grep -v amdgpu.ids | tee gpurun_out/${TAG}_kind_$N.log
  ZT_LIB=$L timeout -k 10 300 python bench.py --no-cpu-baseline --no-api > gpurun_out/${TAG}_bench_$N.log 2>&1
  echo "[$N] $(tail -n 1 gpurun_out/${TAG}_bench_$N.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print({k: d[k] for k in ["value","ms_per_step","match_kernel_ms","deflate_pipeline_ms","inflate_kernel_ms","ratio"]})')"
done
