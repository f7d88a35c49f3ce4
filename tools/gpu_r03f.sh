#!/bin/bash
# Round 3, box 6: the pipelined match kernel (match_kernel_p) -- deflate tests,
# ratio gate and bench against the barrier kernel (ZT_DF_MATCH=barrier); the
# checksum kernel variants.
set -e
TAG=${1:-r03f}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_deflate.py \
  > gpurun_out/${TAG}_pytest.log 2>&1 || { tail -40 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -1 gpurun_out/${TAG}_pytest.log
timeout -k 10 300 python3 tools/ratio_gate.py "" > gpurun_out/${TAG}_gate_p.log 2>&1 && echo "pipelined $(grep '^\[' gpurun_out/${TAG}_gate_p.log)"
ZT_DF_MATCH=barrier timeout -k 10 300 python3 tools/ratio_gate.py "" > gpurun_out/${TAG}_gate_b.log 2>&1 && echo "barrier $(grep '^\[' gpurun_out/${TAG}_gate_b.log)"
timeout -k 10 300 python bench.py --no-cpu-baseline --no-api > gpurun_out/${TAG}_bench_p.log 2>&1
echo "pipelined $(tail -1 gpurun_out/${TAG}_bench_p.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["match_kernel_ms"], d["deflate_pipeline_ms"], d["ratio"])')"
ZT_DF_MATCH=barrier timeout -k 10 300 python bench.py --no-cpu-baseline --no-api > gpurun_out/${TAG}_bench_b.log 2>&1
echo "barrier $(tail -1 gpurun_out/${TAG}_bench_b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["match_kernel_ms"], d["deflate_pipeline_ms"], d["ratio"])')"
for v in "" ck_m3 ck_r32 ck_m3r32; do
  if [ -z "$v" ]; then L=""; else L=$PWD/zlib.ts_amd/build/exp_$v/libzt.so; fi
  echo "[$v] $(ZT_LIB=$L timeout -k 10 120 python tools/ck_time.py 2>&1 | grep checksums)"
done
