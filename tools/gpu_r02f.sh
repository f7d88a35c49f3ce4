#!/bin/bash
# General inflate timing + batch (C4) tests and measurement.  usage: tools/gpu_r02f.sh TAG
TAG=${1:-r02f}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_batch.py -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_batch_t.log 2>&1
rc=$?
grep -E "PASS|FAIL|passed|failed" gpurun_out/${TAG}_batch_t.log | tail -15
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 600 python -u tools/inflate_general_time.py 64 gpurun_out/${TAG}_gen_time.json > gpurun_out/${TAG}_gen_time.log 2>&1 || { tail -20 gpurun_out/${TAG}_gen_time.log; exit 1; }
tail -4 gpurun_out/${TAG}_gen_time.log
timeout -k 10 900 python -u tools/c4_batch.py 10000 gpurun_out/${TAG}_c4.json > gpurun_out/${TAG}_c4.log 2>&1 || { tail -20 gpurun_out/${TAG}_c4.log; exit 1; }
tail -4 gpurun_out/${TAG}_c4.log
