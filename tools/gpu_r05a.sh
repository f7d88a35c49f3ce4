#!/bin/bash
# round 5, first call: paired-ring match kernel (identity digests against the
# dword ring at the same bucket count), GPU tests of this round's changes,
# A/B of the ring layouts / bucket counts, host-API inflate pipeline A/B
set -e
O=gpurun_out/r05a; mkdir -p $O
ZT_LIB=$PWD/zlib.ts_amd/build/r05_ring4h4k/libzt.so timeout -k 10 300 python3 tools/df_digest.py wordsalad mixed > $O/dig_ring4h4k.log 2>&1
timeout -k 10 300 python3 tools/df_digest.py wordsalad mixed > $O/dig_main.log 2>&1
paste -d'|' <(cut -c1-40 $O/dig_ring4h4k.log) <(cut -c1-60 $O/dig_main.log)
TAG=r05a TESTS="tests/test_gpu_deflate.py tests/test_gpu_classify.py tests/test_gpu_ratio.py tests/test_gpu_api_pipeline.py tests/test_gpu_inflate.py" tools/gpu_libab.sh main build/r05_ring4 build/r05_h5k
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_api.log 2>&1
ZT_INF_NOPIPE=1 timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_api_nopipe.log 2>&1
for f in bench_api bench_api_nopipe; do tail -1 $O/$f.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d.get("api"))'; done
