#!/bin/bash
# find_syncs: per-workgroup gathered candidates (one global atomic per
# workgroup) vs per-candidate atomics (ref); spans per workgroup (fs16)
set -e
bash tools/gpu_kab.sh fsv ref=zlib.ts_amd/build/var_ref/libzt.so new=new fs16=zlib.ts_amd/build/var_fs16/libzt.so > gpurun_out/fsv.log 2>&1
for f in ref new fs16; do echo "$f $(grep -h 'find_syncs' gpurun_out/fsv/$f/run_kernel_stats.csv | awk -F'",' '{print $2}' | cut -d, -f1-3) $(grep -h '"value"' gpurun_out/fsv/$f.log | cut -c1-120)"; done
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_inflate.py tests/test_gpu_inflate_general.py tests/test_gpu_api_pipeline.py tests/test_gpu_containers.py > gpurun_out/fsv_pytest.log 2>&1 || { tail -30 gpurun_out/fsv_pytest.log; exit 1; }
tail -1 gpurun_out/fsv_pytest.log
