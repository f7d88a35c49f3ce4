#!/bin/bash
# Round 3: tokenizer pass 2 decodes the marked tokens independently (4 at a time, 16-byte stores): inflate tests, A/B bench and kernel splits, phase cycles
set -e
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=${1:-r03y}
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_inflate.py tests/test_gpu_inflate_general.py tests/test_gpu_batch.py tests/test_gpu_c2.py tests/test_gpu_stream.py \
  > gpurun_out/${TAG}_pytest.log 2>&1 || { tail -40 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -n 1 gpurun_out/${TAG}_pytest.log
for L in "" $R/zlib.ts_amd/build/exp_tkseq/libzt.so; do
  ZT_LIB=$L timeout -k 10 300 python bench.py --no-cpu-baseline --no-api > gpurun_out/${TAG}_bench.log 2>&1
  echo "[${L:+sequential-pass2}] $(tail -n 1 gpurun_out/${TAG}_bench.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print({k: d[k] for k in ["value","ms_per_step","deflate_pipeline_ms","inflate_kernel_ms","inflate_tokenize_ms"]})')"
done
ZT_LIB=$R/zlib.ts_amd/build/exp_tktime/libzt.so timeout -k 10 300 python tools/tk_time.py 256 2>&1 | grep -v amdgpu.ids | tee gpurun_out/${TAG}_tktime.log
ZT_LIB=$R/zlib.ts_amd/build/exp_rs512/libzt.so timeout -k 10 300 python bench.py --no-cpu-baseline --no-api > gpurun_out/${TAG}_bench_rs512.log 2>&1
echo "[expand ring 512] $(tail -n 1 gpurun_out/${TAG}_bench_rs512.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print({k: d[k] for k in ["value","ms_per_step","deflate_pipeline_ms","inflate_kernel_ms","inflate_tokenize_ms"]})')"
cd /tmp
for L in "" $R/zlib.ts_amd/build/exp_rs512/libzt.so; do
  N=${L:+rs512}; N=${N:-intree}
  ZT_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/${TAG}_prof_$N -o run -- python3 $R/bench.py --no-cpu-baseline --no-api --steps 3 > $R/gpurun_out/${TAG}_prof_$N.log 2>&1
  echo "[$N] $(grep -E 'tokenize_kernel|expand_kernel|copy_kernel' $R/gpurun_out/${TAG}_prof_$N/run_kernel_stats.csv | cut -d, -f1,4 | sed 's/zt::(anonymous namespace):://' | tr '\n' ' ')"
done
cd $R
