set -e
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/t2.log 2>&1 || { tail -40 gpurun_out/t2.log; exit 1; }
tail -1 gpurun_out/t2.log
timeout -k 10 600 python tools/bench_configs.py 2>&1 | grep -v amdgpu.ids
