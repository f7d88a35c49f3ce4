#!/bin/bash
# match search: positions of a thread walked one after another, each carrying
# the previous one's match (var_seq) vs two walks interleaved (in-tree):
# deflate tests on the variant, 16-window gate, bench
set -e
R=$GRAFT_REPO_ROOT; mkdir -p gpurun_out/r04s
ZT_LIB=$R/zlib.ts_amd/build/var_seq/libzt.so timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_deflate.py tests/test_gpu_classify.py \
  > gpurun_out/r04s/pytest.log 2>&1 || { tail -30 gpurun_out/r04s/pytest.log; exit 1; }
tail -1 gpurun_out/r04s/pytest.log
for spec in pair=zlib.ts_amd/libzt.so seq=zlib.ts_amd/build/var_seq/libzt.so pair2=zlib.ts_amd/libzt.so seq2=zlib.ts_amd/build/var_seq/libzt.so; do
  name=${spec%%=*}; export ZT_LIB=$R/${spec#*=}
  case $name in *2) ;; *) timeout -k 10 300 python tools/ratio_gate.py > gpurun_out/r04s/gate_$name.log 2>&1 ;; esac
  timeout -k 10 300 python bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-api > gpurun_out/r04s/bench_$name.log 2>&1
  echo "[$name] $(grep '\[' gpurun_out/r04s/gate_${name%2}.log | sed 's/.*\] //' | cut -c1-170) | bench $(tail -1 gpurun_out/r04s/bench_$name.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["match_kernel_ms"], d["ratio"])')"
done
