#!/bin/bash
# Round 3, box 2: r03a's tests + the deflate / inflate suites after the
# DEFLATE-block grouping (ZT_DF_GROUP), the ratio gate, a bench line and the
# bench's kernel stats; the C2 host-API rate and kernel stats.
#   usage: tools/gpu_r03b.sh TAG
set -e
TAG=${1:-r03b}
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_c2.py \
  "tests/test_gpu_batch.py::test_alias_devices_split" tests/test_gpu_zip.py tests/test_gpu_stream.py \
  tests/test_gpu_containers.py tests/test_gpu_deflate.py tests/test_gpu_inflate.py tests/test_gpu_ratio.py \
  tests/test_gpu_batch.py -s > gpurun_out/${TAG}_pytest.log 2>&1 || { tail -60 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -2 gpurun_out/${TAG}_pytest.log
grep -hE "C2:|ratio|^wordsalad|^source|^structured|^xorshift" gpurun_out/${TAG}_pytest.log | head -30 || true
timeout -k 10 300 python3 tools/ratio_gate.py "" "24,128,1,128,8,16,16,1" "20,128,1,128,8,16,16,1" "32,128,1,32,8,16,16,1" "32,128,1,64,8,16,8,1" "24,128,1,64,8,16,8,1" > gpurun_out/${TAG}_gate.log 2>&1
grep '^\[' gpurun_out/${TAG}_gate.log
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/${TAG}_bench.log 2>&1
tail -1 gpurun_out/${TAG}_bench.log
ZT_BATCH_TIMING=1 timeout -k 10 300 python tools/c2_bench.py 5 > gpurun_out/${TAG}_c2.json 2> gpurun_out/${TAG}_c2_stages.log
cat gpurun_out/${TAG}_c2.json
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/${TAG}_c2prof -o run -- python3 $R/tools/c2_bench.py 5 > $R/gpurun_out/${TAG}_c2prof.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/${TAG}_prof -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-api > $R/gpurun_out/${TAG}_prof.log 2>&1
cd $R
cp gpurun_out/${TAG}_c2prof/run_kernel_stats.csv gpurun_out/${TAG}_c2_kernel_stats.csv
cp gpurun_out/${TAG}_prof/run_kernel_stats.csv gpurun_out/${TAG}_kernel_stats.csv
cut -d, -f1-4 gpurun_out/${TAG}_c2_kernel_stats.csv | head -12
cut -d, -f1-4 gpurun_out/${TAG}_kernel_stats.csv | head -14
