#!/bin/bash
# Round 3: tiny deflates through the pipelined match kernel first (bounded), then the A/B of gpu_r03f.sh
set -e
mkdir -p gpurun_out
timeout -k 5 60 python tools/mp_tiny.py > gpurun_out/r03g_tiny.log 2>&1 || { echo "tiny rc $?"; cat gpurun_out/r03g_tiny.log; exit 1; }
grep '^n ' gpurun_out/r03g_tiny.log
bash tools/gpu_r03f.sh r03g
