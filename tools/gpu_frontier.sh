#!/bin/bash
# Ratio / match-time frontier: the 16-window gate (tools/ratio_gate.py) for
# the in-tree build and zlib.ts_amd/build/exp_b64 (64 KiB blocks) at several
# chain depths.   usage: tools/gpu_frontier.sh TAG
set -e
TAG=${1:-fr}
mkdir -p gpurun_out
P="32,128,1,128,8,16,16,1 28,128,1,128,8,16,16,1 24,128,1,128,8,16,16,1 32,128,1,32,8,16,16,1 32,128,1,16,8,16,16,1"
timeout -k 10 300 python3 tools/ratio_gate.py $P > gpurun_out/${TAG}_b32.log 2>&1
ZT_LIB=$PWD/zlib.ts_amd/build/exp_b64/libzt.so timeout -k 10 300 python3 tools/ratio_gate.py $P > gpurun_out/${TAG}_b64.log 2>&1
grep -h '^\[' gpurun_out/${TAG}_b32.log gpurun_out/${TAG}_b64.log
