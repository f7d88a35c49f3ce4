#!/bin/bash
# Phase maps scoped to the sync-point / batch tokenizer: GPU tests, C2, general inflate, bench.
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/p2_tests.log 2>&1 || { tail -30 gpurun_out/p2_tests.log; exit 1; }
tail -1 gpurun_out/p2_tests.log
timeout -k 10 300 python -u tools/c2_kind.py > gpurun_out/p2_c2kind.log 2>&1; grep xorshift gpurun_out/p2_c2kind.log
timeout -k 10 300 python -u tools/c2_probe.py > gpurun_out/p2_c2probe.log 2>&1; grep "count 4096" gpurun_out/p2_c2probe.log
timeout -k 10 600 python -u tools/inflate_general_time.py 64 gpurun_out/p2_gen.json > gpurun_out/p2_gen.log 2>&1
python3 -c "import json; d=json.load(open('gpurun_out/p2_gen.json')); print([(k, v['device']['wall_ms']) for k,v in d.items() if isinstance(v,dict)])"
timeout -k 10 300 python bench.py --no-cpu-baseline --no-api > gpurun_out/p2_bench.log 2>&1
tail -1 gpurun_out/p2_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['inflate_kernel_ms'], d['inflate_tokenize_ms'])"
