#!/bin/bash
# round 5: the host-API paths with their alternatives switched on -- no host
# output pool (ZT_HOST_POOL_MB=0), the one-call inflate (ZT_INF_NOPIPE=1),
# 4 and 16 inflate pieces -- over the API / container / batch / stream suites
set -e
O=gpurun_out/r05ac; mkdir -p $O; export TMPDIR=/tmp
T="tests/test_gpu_api_pipeline.py tests/test_gpu_containers.py tests/test_gpu_zip.py tests/test_gpu_stream.py tests/test_gpu_batch.py tests/test_gpu_inflate.py"
for e in ZT_HOST_POOL_MB=0 ZT_INF_NOPIPE=1 ZT_INF_PIECES=4 ZT_INF_PIECES=16; do
  env $e timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread $T > $O/pytest_$e.log 2>&1 || { echo "$e FAILED"; tail -20 $O/pytest_$e.log; exit 1; }
  echo "$e: $(tail -1 $O/pytest_$e.log)"
done
