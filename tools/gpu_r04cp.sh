#!/bin/bash
# copy step 512 (in-tree) vs 1024 bytes (build/var_cp1024): inflate tests on
# the variant, bench inflate split, interleaved A/B
set -e
TAG=${1:-r04cp}
R=$GRAFT_REPO_ROOT; mkdir -p gpurun_out/$TAG
ZT_LIB=$R/zlib.ts_amd/build/var_cp1024/libzt.so timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_inflate.py tests/test_gpu_inflate_general.py tests/test_gpu_stored_runs.py tests/test_gpu_c2.py tests/test_gpu_batch.py tests/test_gpu_stream.py \
  > gpurun_out/$TAG/pytest.log 2>&1 || { tail -30 gpurun_out/$TAG/pytest.log; exit 1; }
tail -1 gpurun_out/$TAG/pytest.log
for spec in s512=zlib.ts_amd/libzt.so s1024=zlib.ts_amd/build/var_cp1024/libzt.so s512b=zlib.ts_amd/libzt.so s1024b=zlib.ts_amd/build/var_cp1024/libzt.so; do
  name=${spec%%=*}; export ZT_LIB=$R/${spec#*=}
  timeout -k 10 300 python bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-api > gpurun_out/$TAG/bench_$name.log 2>&1
  echo "[$name] $(tail -n 1 gpurun_out/$TAG/bench_$name.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print({k: d.get(k) for k in ["value","inflate_kernel_ms","inflate_tokenize_ms"]})')"
done
export TMPDIR=/tmp
for spec in s512=zlib.ts_amd/libzt.so s1024=zlib.ts_amd/build/var_cp1024/libzt.so; do
  name=${spec%%=*}; export ZT_LIB=$R/${spec#*=}
  cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/$TAG/prof_$name -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-api > $R/gpurun_out/$TAG/prof_$name.log 2>&1
  cd $R
  echo "[$name] $(grep -E 'expand_kernel|copy_kernel' gpurun_out/$TAG/prof_$name/run_kernel_stats.csv | cut -d, -f1,4 | sed 's/zt::(anonymous namespace):://' | tr '\n' ' ')"
done
