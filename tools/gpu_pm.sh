#!/bin/bash
# Fused post-match kernel: deflate tests, ratio gate, bench fused (4 and 3 waves per SIMD) vs unfused
set -e
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=${1:-pm}
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_deflate.py tests/test_gpu_ratio.py \
  > gpurun_out/${TAG}_pytest.log 2>&1 || { tail -30 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -n 1 gpurun_out/${TAG}_pytest.log
timeout -k 10 300 python3 tools/ratio_gate.py "" > gpurun_out/${TAG}_gate.log 2>&1 && grep '^\[' gpurun_out/${TAG}_gate.log
for cfg in "fused4::" "fused3:$R/zlib.ts_amd/build/exp_pm3/libzt.so:" "unfused::1"; do
  N=${cfg%%:*}; rest=${cfg#*:}; L=${rest%%:*}; U=${rest#*:}
  ZT_DF_UNFUSED=$U ZT_LIB=$L timeout -k 10 300 python bench.py --no-cpu-baseline --no-api > gpurun_out/${TAG}_bench_$N.log 2>&1
  echo "[$N] $(tail -n 1 gpurun_out/${TAG}_bench_$N.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print({k: d[k] for k in ["value","ms_per_step","match_kernel_ms","deflate_pipeline_ms","inflate_kernel_ms","ratio"]})')"
done
