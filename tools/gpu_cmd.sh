set -e
timeout -k 10 600 python bench.py --steps 3 > gpurun_out/b3.log 2>&1
grep -v amdgpu.ids gpurun_out/b3.log | tail -2
