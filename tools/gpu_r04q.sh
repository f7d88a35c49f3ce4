#!/bin/bash
# Phase maps decoded 4 start phases at a time and recomposed after every
# repair (in-tree) vs the round-3 maps (build/var_pri8: HEAD with ZT_PRI=8);
# fused checksum merge (in-tree) vs the separate finish kernel (var_pri8).
#   usage: tools/gpu_r04q.sh TAG
set -e
TAG=${1:-r04q}
R=$GRAFT_REPO_ROOT; mkdir -p gpurun_out/$TAG; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_inflate.py tests/test_gpu_inflate_general.py tests/test_gpu_stored_runs.py tests/test_gpu_c2.py tests/test_gpu_batch.py tests/test_gpu_checksums.py tests/test_gpu_containers.py \
  > gpurun_out/$TAG/pytest.log 2>&1 || { tail -30 gpurun_out/$TAG/pytest.log; exit 1; }
tail -1 gpurun_out/$TAG/pytest.log
for spec in old=zlib.ts_amd/build/var_pri8/libzt.so new=zlib.ts_amd/libzt.so pm3=zlib.ts_amd/build/var_pm3/libzt.so pm5=zlib.ts_amd/build/var_pm5/libzt.so; do
  name=${spec%%=*}; export ZT_LIB=$R/${spec#*=}
  cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/$TAG/c2_$name -o run -- python3 $R/tools/c2_bench.py 3 > $R/gpurun_out/$TAG/c2_$name.log 2>&1
  timeout -k 10 180 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/$TAG/ck_$name -o run -- python3 $R/tools/ck_time.py > $R/gpurun_out/$TAG/ck_$name.log 2>&1
  cd $R
  echo "[$name C2] $(tail -1 gpurun_out/$TAG/c2_$name.log | cut -c1-200)"
  echo "[$name C2] $(grep -E 'tokenize_kernel|expand_kernel|copy_kernel' gpurun_out/$TAG/c2_$name/run_kernel_stats.csv | cut -d, -f1,3,4 | sed 's/zt::(anonymous namespace):://' | tr '\n' ' ')"
  echo "[$name C1] $(grep -E 'checksum' gpurun_out/$TAG/ck_$name/run_kernel_stats.csv | cut -d, -f1-4,6,7 | sed 's/zt::(anonymous namespace):://' | cut -c1-30,100- | tr '\n' ' ')"
  timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-api > gpurun_out/$TAG/bench_$name.log 2>&1
  echo "[$name] $(tail -n 1 gpurun_out/$TAG/bench_$name.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print({k: d.get(k) for k in ["value","deflate_pipeline_ms","inflate_kernel_ms","inflate_tokenize_ms"]})')"
done
for spec in old=zlib.ts_amd/build/var_pri8tk/libzt.so new=zlib.ts_amd/build/var_tktime/libzt.so; do
  name=${spec%%=*}; export ZT_LIB=$R/${spec#*=}
  timeout -k 10 300 python3 tools/c2_tk_time.py 512 > gpurun_out/$TAG/c2_tk_$name.log 2>&1
  echo "[$name]"; grep -v amdgpu.ids gpurun_out/$TAG/c2_tk_$name.log
done
