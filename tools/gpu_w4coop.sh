#!/bin/bash
# 4 walks per lane + cooperative candidate measurement (build/var_w4,
# -DZT_DF_WALK4=1) vs the in-tree build: 16-window ratio gate at several
# chain depths, then the deflate parity tests on the variant.
set -e
mkdir -p gpurun_out/w4
timeout -k 10 300 python3 -u tools/ratio_gate.py "" > gpurun_out/w4/gate_base.log 2>&1
ZT_LIB=$PWD/zlib.ts_amd/build/var_w4/libzt.so timeout -k 10 600 python3 -u tools/ratio_gate.py "" "28,128,1,128,8,16,16,1" "24,128,1,128,8,16,16,1" "20,128,1,128,8,16,16,1" "16,128,1,128,8,16,16,1" > gpurun_out/w4/gate_w4.log 2>&1
grep -v amdgpu.ids gpurun_out/w4/gate_base.log gpurun_out/w4/gate_w4.log
ZT_LIB=$PWD/zlib.ts_amd/build/var_w4/libzt.so timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_deflate.py > gpurun_out/w4/pytest.log 2>&1 || { tail -30 gpurun_out/w4/pytest.log; exit 1; }
tail -3 gpurun_out/w4/pytest.log
