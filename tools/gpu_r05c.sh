#!/bin/bash
# round 5, third call: the step's four reads joined (one LDS round trip per
# hop), candidate measurement deferred to every second step, their
# combination with u16 heads -- identical-stream digests + match times; C1
# checksum kernel with LDS-staged rows; the GPU tests of this round's changes
set -e
O=gpurun_out/r05c; mkdir -p $O
for L in main r05_join r05_defer r05_jd r05_jdh16 main; do
  if [ $L = main ]; then unset ZT_LIB; else export ZT_LIB=$PWD/zlib.ts_amd/build/$L/libzt.so; fi
  DF_LEVELS=6 timeout -k 10 200 python3 tools/df_digest.py wordsalad structured mixed > $O/dig_$L.log 2>&1
  echo "$L $(grep L6 $O/dig_$L.log | awk '{printf "%s %s %s %s | ", $2, $3, $5, $7}')"
done
for L in main r05_ckst main r05_ckst; do
  if [ $L = main ]; then unset ZT_LIB; else export ZT_LIB=$PWD/zlib.ts_amd/build/$L/libzt.so; fi
  timeout -k 10 120 python3 tools/ck_time.py > $O/ck_$L.log 2>&1; echo "$L $(tail -1 $O/ck_$L.log)"
done
export ZT_LIB=$PWD/zlib.ts_amd/build/r05_ckst/libzt.so
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_checksums.py > $O/pytest_ck.log 2>&1 || { tail -30 $O/pytest_ck.log; exit 1; }
tail -1 $O/pytest_ck.log
unset ZT_LIB
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_api_pipeline.py tests/test_gpu_inflate.py tests/test_gpu_deflate.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_api.log 2>&1
ZT_INF_NOPIPE=1 timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_api_nopipe.log 2>&1
for f in bench_api bench_api_nopipe; do tail -1 $O/$f.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["match_kernel_ms"], d.get("api"))'; done
