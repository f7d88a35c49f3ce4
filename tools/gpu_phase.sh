#!/bin/bash
# Phase-map check: GPU tests, C2 latency per corpus / batch size, bench.
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/ph_tests.log 2>&1 || { tail -30 gpurun_out/ph_tests.log; exit 1; }
tail -1 gpurun_out/ph_tests.log
timeout -k 10 300 python -u tools/c2_kind.py > gpurun_out/ph_c2kind.log 2>&1; grep -v amdgpu gpurun_out/ph_c2kind.log | tail -8
timeout -k 10 300 python -u tools/c2_probe.py > gpurun_out/ph_c2probe.log 2>&1; grep -v amdgpu gpurun_out/ph_c2probe.log | tail -6
timeout -k 10 300 python bench.py --no-cpu-baseline --no-api > gpurun_out/ph_bench.log 2>&1; tail -1 gpurun_out/ph_bench.log | cut -c 560-760
