set -e
timeout -k 10 600 python -m pytest tests -m gpu -x -q -k deflate > gpurun_out/t2.log 2>&1 || { tail -40 gpurun_out/t2.log; exit 1; }
tail -1 gpurun_out/t2.log
timeout -k 10 600 python tools/df_sweep.py xorshift32 32,128,1,128,8,16,16 1,128,1,128,8,0,16 2>&1 | grep -v amdgpu.ids
timeout -k 10 600 python tools/df_sweep.py wordsalad 32,128,1,128,8,16,16 2>&1 | grep -v amdgpu.ids
timeout -k 10 600 python bench.py --steps 3 --no-cpu-baseline > gpurun_out/b5.log 2>&1
grep -v amdgpu.ids gpurun_out/b5.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: d[k] for k in ['value','ratio','match_kernel_ms','deflate_pipeline_ms','inflate_kernel_ms','inflate_tokenize_ms']})"
