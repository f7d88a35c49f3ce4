#!/bin/bash
# round 5, second call: ds_mskor lane order (u16 chain heads), marginal LDS
# cost of one more link / filter / extension read per event (identical
# streams), bucket-count variants on the ratio gate, then the GPU tests of
# this round's changes and the host-API inflate pipeline A/B
set -e
O=gpurun_out/r05b; mkdir -p $O
timeout -k 5 60 tools/micro/lds_mskor_order > $O/mskor.log 2>&1; tail -1 $O/mskor.log
for L in main r05_xlink r05_xfilt r05_xext r05_h16 r05_h4k main; do
  if [ $L = main ]; then unset ZT_LIB; else export ZT_LIB=$PWD/zlib.ts_amd/build/$L/libzt.so; fi
  DF_LEVELS=6 timeout -k 10 200 python3 tools/df_digest.py wordsalad structured mixed > $O/dig_$L.log 2>&1
  echo "$L $(grep L6 $O/dig_$L.log | awk '{printf "%s %s %s %s | ", $2, $3, $5, $7}')"
done
for L in main r05_h16 r05_h4k; do
  if [ $L = main ]; then unset ZT_LIB; else export ZT_LIB=$PWD/zlib.ts_amd/build/$L/libzt.so; fi
  timeout -k 10 300 python tools/ratio_gate.py > $O/gate_$L.log 2>&1
  echo "$L $(grep -o 'wordsalad [0-9.]*.*' $O/gate_$L.log)"
done
unset ZT_LIB
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ratio.py tests/test_gpu_classify.py tests/test_gpu_deflate.py tests/test_gpu_api_pipeline.py tests/test_gpu_inflate.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_api.log 2>&1
ZT_INF_NOPIPE=1 timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_api_nopipe.log 2>&1
for f in bench_api bench_api_nopipe; do tail -1 $O/$f.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["match_kernel_ms"], d.get("api"))'; done
