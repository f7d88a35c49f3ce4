#!/bin/bash
# Config C2 (4096 reference-deflated 64 KiB blocks) device kernel times for
# two builds (rocprofv3 kernel stats of tools/c2_bench.py) + the C2 test.
set -e
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out/c2ab
export TMPDIR=/tmp
for spec in ref=zlib.ts_amd/build/var_ref/libzt.so new=new; do
  name=${spec%%=*}; lib=${spec#*=}
  if [ "$lib" = new ]; then unset ZT_LIB; else export ZT_LIB=$R/$lib; fi
  cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/c2ab/$name -o run -- python3 $R/tools/c2_bench.py 5 > $R/gpurun_out/c2ab/$name.log 2>&1
  cd $R
  echo "== $name $(tail -1 gpurun_out/c2ab/$name.log | cut -c1-300)"
  cut -d, -f1-4 gpurun_out/c2ab/$name/run_kernel_stats.csv | head -8
done
unset ZT_LIB
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_c2.py tests/test_gpu_inflate.py tests/test_gpu_zip.py tests/test_gpu_containers.py > gpurun_out/c2ab/pytest.log 2>&1 || { tail -30 gpurun_out/c2ab/pytest.log; exit 1; }
tail -1 gpurun_out/c2ab/pytest.log
