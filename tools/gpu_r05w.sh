#!/bin/bash
# round 5: where a match workgroup's wave cycles go at HEAD (-DZT_DF_TIME
# build, tools/df_time.py): hash phase, serial link, link waits, search,
# idle at the sub-chunk barrier, per wave and 4 KiB sub-chunk
set -e
O=gpurun_out/r05w; mkdir -p $O; export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
ZT_LIB=$R/zlib.ts_amd/build/r05_dftime/libzt.so timeout -k 10 300 python3 tools/df_time.py wordsalad structured mixed > $O/time.log 2>&1
grep -v amdgpu.ids $O/time.log
