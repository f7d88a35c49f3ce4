#!/bin/bash
# encode_kernel: block words staged in LDS and flushed coalesced (in-tree) vs
# stored straight from each thread (var_enc0): deflate tests, kernel stats,
# WRITE_SIZE / read requests of one bench step
set -e
TAG=${1:-r04enc}
R=$GRAFT_REPO_ROOT; mkdir -p gpurun_out/$TAG; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_deflate.py tests/test_gpu_classify.py tests/test_gpu_api_pipeline.py tests/test_gpu_batch.py tests/test_gpu_containers.py \
  > gpurun_out/$TAG/pytest.log 2>&1 || { tail -30 gpurun_out/$TAG/pytest.log; exit 1; }
tail -1 gpurun_out/$TAG/pytest.log
for spec in cache=zlib.ts_amd/libzt.so lds=zlib.ts_amd/build/var_enc1/libzt.so direct=zlib.ts_amd/build/var_enc0/libzt.so; do
  name=${spec%%=*}; export ZT_LIB=$R/${spec#*=}
  cd /tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/$TAG/prof_$name -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-api > $R/gpurun_out/$TAG/prof_$name.log 2>&1
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -f csv -d $R/gpurun_out/$TAG/w_$name -o run -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-api > $R/gpurun_out/$TAG/w_$name.log 2>&1
  cd $R
  echo "[$name] encode $(grep -E 'encode_kernel' gpurun_out/$TAG/prof_$name/run_kernel_stats.csv | cut -d, -f4) ns; WRITE_SIZE $(python3 -c "
import csv,collections
t=collections.defaultdict(float); n=collections.defaultdict(set)
for r in csv.DictReader(open('gpurun_out/$TAG/w_$name/run_counter_collection.csv')):
    if 'encode_kernel' in r['Kernel_Name']: t[0]+=float(r['Counter_Value']); n[0].add(r['Dispatch_Id'])
print(round(t[0]*1024/max(1,len(n[0]))/1e9,3), 'GB per launch')")"
done
# checksum merge: two-level sharded atomics (in-tree) vs one accumulator (var_ckold)
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_checksums.py tests/test_gpu_containers.py > gpurun_out/$TAG/pytest_ck.log 2>&1 || { tail -30 gpurun_out/$TAG/pytest_ck.log; exit 1; }
tail -1 gpurun_out/$TAG/pytest_ck.log
for spec in sharded=zlib.ts_amd/libzt.so one=zlib.ts_amd/build/var_ckold/libzt.so sharded2=zlib.ts_amd/libzt.so one2=zlib.ts_amd/build/var_ckold/libzt.so; do
  name=${spec%%=*}; export ZT_LIB=$R/${spec#*=}
  cd /tmp && timeout -k 10 180 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/$TAG/ck_$name -o run -- python3 $R/tools/ck_time.py > $R/gpurun_out/$TAG/ck_$name.log 2>&1
  cd $R
  echo "[$name] $(python3 -c "
import csv
for r in csv.DictReader(open('gpurun_out/$TAG/ck_$name/run_kernel_stats.csv')):
    if 'checksum' in r['Name']: print(r['Name'][24:44], r['AverageNs'], r['MinNs'])
" | tr '\n' ' ')"
done
# match kernel key hashing: four positions per thread (in-tree) vs one (var_hash1)
for spec in quad=zlib.ts_amd/libzt.so one=zlib.ts_amd/build/var_hash1/libzt.so quad2=zlib.ts_amd/libzt.so one2=zlib.ts_amd/build/var_hash1/libzt.so; do
  name=${spec%%=*}; export ZT_LIB=$R/${spec#*=}
  timeout -k 10 300 python bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-api > gpurun_out/$TAG/bench_$name.log 2>&1
  echo "[$name] $(tail -n 1 gpurun_out/$TAG/bench_$name.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print({k: d.get(k) for k in ["value","match_kernel_ms","deflate_pipeline_ms","inflate_kernel_ms","ratio"]})')"
done
