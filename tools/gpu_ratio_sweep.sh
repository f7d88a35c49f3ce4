#!/bin/bash
# Ratio gate (16 windows) for level-6 parameter variants: ratio vs reference
# per generator and match time.   usage: tools/gpu_ratio_sweep.sh TAG "params" ...
TAG=$1; shift
mkdir -p gpurun_out
timeout -k 10 500 python3 tools/ratio_gate.py "" "$@" > gpurun_out/${TAG}.log 2>&1
cat gpurun_out/${TAG}.log | grep -v amdgpu.ids
