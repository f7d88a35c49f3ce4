#!/bin/bash
# Round 3: checksum kernel (32-row segments, table load only where a ragged
# segment needs it) tests + rocprof; per-generator deflate / inflate times.
set -e
R=$GRAFT_REPO_ROOT
bash tools/gpu_ck_var.sh r03i -
timeout -k 10 300 python tools/kind_time.py 256 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r03i_kind.log
ZT_LIB=$R/zlib.ts_amd/build/exp_tok_simple/libzt.so timeout -k 10 300 python tools/kind_time.py 256 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r03i_kind_simple.log
