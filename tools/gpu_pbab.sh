#!/bin/bash
# parse / price staging ring of 3 chunks (build/exp_pb3: 5.1 KiB LDS) vs 4 (in-tree): deflate tests, rocprof of the bench
set -e
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
ZT_LIB=$R/zlib.ts_amd/build/exp_pb3/libzt.so timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_deflate.py > gpurun_out/${1}_pytest.log 2>&1 || { tail -30 gpurun_out/${1}_pytest.log; exit 1; }
tail -n 1 gpurun_out/${1}_pytest.log
cd /tmp
for rep in 1 2; do
for L in "" $R/zlib.ts_amd/build/exp_pb3/libzt.so; do
  N=${L:+pb3}; N=${N:-intree}
  ZT_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/${1}_prof_$N -o run -- python3 $R/bench.py --no-cpu-baseline --no-api --steps 5 > $R/gpurun_out/${1}_prof_$N.log 2>&1
  echo "[$N] $(grep -E 'parse_kernel|price_kernel' $R/gpurun_out/${1}_prof_$N/run_kernel_stats.csv | cut -d, -f1,4 | sed 's/zt::(anonymous namespace):://' | tr '\n' ' ')"
done
done
