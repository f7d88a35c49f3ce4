#!/bin/bash
# round 5: what the chain walk's measurements find (ZT_DF_COUNT build): the
# share of measured candidates that improve the match, that match fewer than
# 8 bytes (8-byte-key collisions), that gain nothing
set -e
O=gpurun_out/r05r; mkdir -p $O; export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
ZT_LIB=$R/zlib.ts_amd/build/r05_cnt/libzt.so timeout -k 10 300 python3 tools/df_count.py wordsalad structured mixed > $O/count.log 2>&1
cat $O/count.log | grep -v amdgpu.ids
