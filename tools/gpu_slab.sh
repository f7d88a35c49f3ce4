#!/bin/bash
# Slab outputs check: GPU tests, C2 host stages, C4 batch.
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/sl_tests.log 2>&1 || { tail -30 gpurun_out/sl_tests.log; exit 1; }
tail -1 gpurun_out/sl_tests.log
ZT_BATCH_TIMING=1 timeout -k 10 300 python -u tools/c2_probe.py > gpurun_out/sl_c2.log 2>&1; grep -v amdgpu gpurun_out/sl_c2.log | tail -10
timeout -k 10 300 python -u tools/c4_batch.py 10000 gpurun_out/sl_c4.json > gpurun_out/sl_c4.log 2>&1; grep "1 GPU" gpurun_out/sl_c4.log
