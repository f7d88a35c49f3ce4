set -e
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/t2.log 2>&1 || { tail -40 gpurun_out/t2.log; exit 1; }
tail -3 gpurun_out/t2.log
ZT_INF_DEBUG=1 timeout -k 10 600 python bench.py --steps 3 --no-cpu-baseline > gpurun_out/b2.log 2>&1
grep -v amdgpu.ids gpurun_out/b2.log | tail -3
