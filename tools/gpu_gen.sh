#!/bin/bash
# General-inflate iteration on one GPU box: its tests (with fallback reasons
# on stderr), then timing.   usage: tools/gpu_gen.sh TAG [MiB]
TAG=${1:-gen}; MIB=${2:-64}
mkdir -p gpurun_out
export TMPDIR=/tmp
ZT_INF_DEBUG=1 timeout -k 10 900 python -u -m pytest tests/test_gpu_inflate_general.py -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_t.log 2>&1
rc=$?
grep -E "passed|failed|PASS|FAIL|Error|error" gpurun_out/${TAG}_t.log | tail -40
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 600 python -u tools/inflate_general_time.py $MIB gpurun_out/${TAG}_time.json > gpurun_out/${TAG}_time.log 2>&1
rc2=$?
tail -5 gpurun_out/${TAG}_time.log
exit $rc2
