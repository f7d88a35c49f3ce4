set -e
timeout -k 10 600 python -m pytest tests -m gpu -x -q -k deflate > gpurun_out/t2.log 2>&1 || { tail -40 gpurun_out/t2.log; exit 1; }
tail -1 gpurun_out/t2.log
timeout -k 10 600 python tools/df_sweep.py wordsalad 32,128,1,128,8,16,16 2>&1 | grep -v amdgpu.ids
timeout -k 10 600 python tools/df_sweep.py structured 32,128,1,128,8,16,16 2>&1 | grep -v amdgpu.ids
