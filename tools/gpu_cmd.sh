set -e
timeout -k 10 600 python bench.py --steps 3 --no-cpu-baseline > gpurun_out/b5.log 2>&1
grep -v amdgpu.ids gpurun_out/b5.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: d[k] for k in ['value','ratio','match_kernel_ms','deflate_pipeline_ms','inflate_kernel_ms','inflate_tokenize_ms']})"
