#!/bin/bash
# round 5: the SIMT tokenizer's cycle split per round at HEAD (-DZT_TK_TIME
# build, tools/tk_time.py): staging, pass 1, repairs, pass 2
set -e
O=gpurun_out/r05ab; mkdir -p $O; export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
ZT_LIB=$R/zlib.ts_amd/build/r05_tktime/libzt.so timeout -k 10 300 python3 tools/tk_time.py 256 wordsalad structured mixed xorshift32 > $O/tk.log 2>&1
grep -v amdgpu.ids $O/tk.log
