#!/bin/bash
# tokenizer: next round's input loaded before pass 2 (in-tree) vs not (var_pf0)
set -e
TAG=${1:-r04pf}
R=$GRAFT_REPO_ROOT; mkdir -p gpurun_out/$TAG; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_inflate.py tests/test_gpu_inflate_general.py tests/test_gpu_stored_runs.py tests/test_gpu_c2.py tests/test_gpu_batch.py \
  > gpurun_out/$TAG/pytest.log 2>&1 || { tail -30 gpurun_out/$TAG/pytest.log; exit 1; }
tail -1 gpurun_out/$TAG/pytest.log
for spec in pf1=zlib.ts_amd/libzt.so pf0=zlib.ts_amd/build/var_pf0/libzt.so; do
  name=${spec%%=*}; export ZT_LIB=$R/${spec#*=}
  cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/$TAG/prof_$name -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-api > $R/gpurun_out/$TAG/prof_$name.log 2>&1
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/$TAG/c2_$name -o run -- python3 $R/tools/c2_bench.py 3 > $R/gpurun_out/$TAG/c2_$name.log 2>&1
  cd $R
  echo "[$name bench] $(grep -E 'tokenize_kernel' gpurun_out/$TAG/prof_$name/run_kernel_stats.csv | cut -d, -f4)  [C2] $(grep -E 'tokenize_kernel' gpurun_out/$TAG/c2_$name/run_kernel_stats.csv | cut -d, -f4)"
done
