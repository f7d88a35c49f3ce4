#!/bin/bash
# Round 3: expand_kernel with 256-byte windows: inflate tests, bench, A/B against the 64-byte kernel
set -e
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=${1:-r03o}
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_inflate.py tests/test_gpu_inflate_general.py tests/test_gpu_batch.py tests/test_gpu_c2.py tests/test_gpu_stream.py tests/test_gpu_zip.py tests/test_gpu_containers.py \
  > gpurun_out/${TAG}_pytest.log 2>&1 || { tail -40 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -n 1 gpurun_out/${TAG}_pytest.log
for L in "" $R/zlib.ts_amd/build/exp_ex1/libzt.so; do
  ZT_LIB=$L timeout -k 10 300 python bench.py --no-cpu-baseline --no-api > gpurun_out/${TAG}_bench.log 2>&1
  echo "[$L] $(tail -n 1 gpurun_out/${TAG}_bench.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print({k: d[k] for k in ["value","ms_per_step","deflate_pipeline_ms","inflate_kernel_ms","inflate_tokenize_ms"]})')"
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/${TAG}_bprof -o run -- python3 $R/bench.py --no-cpu-baseline --no-api --steps 5 > $R/gpurun_out/${TAG}_bprof.log 2>&1
cd $R
python3 -c "
import csv, re
for r in csv.DictReader(open('gpurun_out/${TAG}_bprof/run_kernel_stats.csv')):
    n = re.split(r'[(<]', r['Name'].replace('zt::(anonymous namespace)::', ''))[0][:28]
    if 'rocprim' in n or 'rocclr' in n or 'at::' in n: continue
    print(f'  {n:28s} {int(r[\"Calls\"]):4d} {float(r[\"AverageNs\"])/1e6:8.3f} ms')
"
