#!/bin/bash
# r02g: general inflate fix check, zip tests, full GPU suite, timing.  usage: tools/gpu_r02g.sh TAG
TAG=${1:-r02g}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/gen_debug.py 64 > gpurun_out/${TAG}_dbg.log 2>&1 || { tail -5 gpurun_out/${TAG}_dbg.log; exit 1; }
grep -E "olen|mismatch|OK" gpurun_out/${TAG}_dbg.log
timeout -k 10 1200 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?
tail -15 gpurun_out/${TAG}_pytest.log | grep -E "passed|failed|FAILED|Error" 
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 600 python -u tools/inflate_general_time.py 64 gpurun_out/${TAG}_gen_time.json > gpurun_out/${TAG}_gen_time.log 2>&1 || { tail -20 gpurun_out/${TAG}_gen_time.log; exit 1; }
grep device gpurun_out/${TAG}_gen_time.log
