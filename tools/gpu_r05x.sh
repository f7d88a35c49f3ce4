#!/bin/bash
# round 5: what a 24 KiB window would cost in ratio (the match kernel's
# distance cap at 24 256 instead of 28 352; a 4 KiB-shorter window is what
# 8 KiB sub-chunks -- half the barriers -- would leave in the 32 KiB ring):
# the 16-window gate of main and of r05_maxd24
set -e
O=gpurun_out/r05x; mkdir -p $O; export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python3 tools/ratio_gate.py > $O/gate_main.log 2>&1; tail -1 $O/gate_main.log
ZT_LIB=$R/zlib.ts_amd/build/r05_maxd24/libzt.so timeout -k 10 300 python3 tools/ratio_gate.py > $O/gate_maxd24.log 2>&1; tail -1 $O/gate_maxd24.log
