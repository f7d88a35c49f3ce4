#!/bin/bash
# Level-6 ratio gate over search-cut variants (skip / nice / good / chain).
set -e
mkdir -p gpurun_out/skip
timeout -k 10 900 python3 -u tools/ratio_gate.py "" "32,128,1,64,8,16,16,1" "32,128,1,48,8,16,16,1" "32,128,1,32,8,16,16,1" "32,128,1,24,8,16,16,1" "32,64,1,64,8,16,16,1" "40,128,1,32,8,16,16,1" "48,128,1,32,8,16,16,1" "32,128,1,32,8,16,24,1" "48,128,1,24,8,16,16,1" > gpurun_out/skip/gate.log 2>&1
grep -v amdgpu.ids gpurun_out/skip/gate.log
