#!/bin/bash
# A/B of the cooperative candidate measurement: digests + match times of
# build/var_ref (ZT_DF_COOP=0) vs the in-tree libzt.so, then the deflate
# parity tests on the in-tree build.   usage: tools/gpu_coop.sh TAG
set -e
TAG=${1:-coop}
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
ZT_LIB=$PWD/zlib.ts_amd/build/var_ref/libzt.so timeout -k 10 300 python3 -u tools/df_digest.py > gpurun_out/$TAG/ref.log 2>&1
timeout -k 10 300 python3 -u tools/df_digest.py > gpurun_out/$TAG/new.log 2>&1
paste -d'|' <(grep ratio gpurun_out/$TAG/ref.log) <(grep ratio gpurun_out/$TAG/new.log | cut -c1-200)
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_deflate.py tests/test_gpu_ratio.py > gpurun_out/$TAG/pytest.log 2>&1 || { tail -30 gpurun_out/$TAG/pytest.log; exit 1; }
tail -5 gpurun_out/$TAG/pytest.log
