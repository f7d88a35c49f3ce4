#!/bin/bash
# Primary decode table bits 7 vs 8 (ZT_PRI): inflate tests on the PRI 8 build,
# bench inflate split, C2 device kernel times and tokenizer phase cycles.
#   usage: tools/gpu_r04_pri.sh TAG
set -e
TAG=${1:-r04pri}
R=$GRAFT_REPO_ROOT; mkdir -p gpurun_out/$TAG; export TMPDIR=/tmp
ZT_LIB=$R/zlib.ts_amd/build/var_pri8/libzt.so timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_inflate.py tests/test_gpu_inflate_general.py tests/test_gpu_stored_runs.py tests/test_gpu_c2.py tests/test_gpu_batch.py \
  > gpurun_out/$TAG/pytest_pri8.log 2>&1 || { tail -30 gpurun_out/$TAG/pytest_pri8.log; exit 1; }
tail -1 gpurun_out/$TAG/pytest_pri8.log
for spec in pri7=zlib.ts_amd/libzt.so pri8=zlib.ts_amd/build/var_pri8/libzt.so; do
  name=${spec%%=*}; export ZT_LIB=$R/${spec#*=}
  timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-api > gpurun_out/$TAG/bench_$name.log 2>&1
  echo "[$name] $(tail -n 1 gpurun_out/$TAG/bench_$name.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print({k: d.get(k) for k in ["value","deflate_pipeline_ms","inflate_kernel_ms","inflate_tokenize_ms"]})')"
  cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/$TAG/c2_$name -o run -- python3 $R/tools/c2_bench.py 3 > $R/gpurun_out/$TAG/c2_$name.log 2>&1
  cd $R
  echo "[$name C2] $(grep -E 'tokenize_kernel|expand_kernel|copy_kernel' gpurun_out/$TAG/c2_$name/run_kernel_stats.csv | cut -d, -f1,3,4 | sed 's/zt::(anonymous namespace):://' | tr '\n' ' ')"
done
for spec in pri7=zlib.ts_amd/build/var_tktime/libzt.so pri8=zlib.ts_amd/build/var_pri8tk/libzt.so; do
  name=${spec%%=*}; export ZT_LIB=$R/${spec#*=}
  timeout -k 10 300 python3 tools/c2_tk_time.py 512 > gpurun_out/$TAG/c2_tk_$name.log 2>&1
  echo "[$name]"; grep -v amdgpu.ids gpurun_out/$TAG/c2_tk_$name.log
done
