set -e
ZT_INF_DEBUG=1 timeout -k 10 300 python tools/inf_debug.py 2>&1 | grep -v amdgpu.ids
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/t2.log 2>&1 || { tail -40 gpurun_out/t2.log; exit 1; }
tail -2 gpurun_out/t2.log
timeout -k 10 600 python tools/inflate_phase_time.py 2>&1 | grep -v amdgpu.ids
timeout -k 10 600 python bench.py --steps 3 --no-cpu-baseline > gpurun_out/b5.log 2>&1
grep -v amdgpu.ids gpurun_out/b5.log | tail -1
