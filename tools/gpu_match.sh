#!/bin/bash
# Match-kernel iteration: ratio gate table (16 windows), deflate digests and
# times on 128 MiB corpora (level 6), then the bench line.   usage: tools/gpu_match.sh TAG
set -e
TAG=${1:-m}
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/ratio_gate.py "" > gpurun_out/${TAG}_gate.log 2>&1; grep level6 gpurun_out/${TAG}_gate.log
timeout -k 10 300 python3 tools/df_digest.py > gpurun_out/${TAG}_dig.log 2>&1; grep L6 gpurun_out/${TAG}_dig.log
timeout -k 10 300 python bench.py --no-cpu-baseline --no-api > gpurun_out/${TAG}_bench.log 2>&1; tail -1 gpurun_out/${TAG}_bench.log | cut -c1-60,700-1000
