#!/bin/bash
# sequential carried walks where a carried match can be replaced by an equally
# long nearer one (ZT_DF_CARRY_TIES): gate + bench per (build, chain)
set -e
R=$GRAFT_REPO_ROOT; mkdir -p gpurun_out/r04s3
ZT_LIB=$R/zlib.ts_amd/build/var_seqt/libzt.so timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_deflate.py \
  > gpurun_out/r04s3/pytest.log 2>&1 || { tail -30 gpurun_out/r04s3/pytest.log; exit 1; }
tail -1 gpurun_out/r04s3/pytest.log
for spec in seqt:28=var_seqt seqt:24=var_seqt seqt:20=var_seqt pairt:28=var_pairt pairt:24=var_pairt; do
  name=${spec%%=*}; ch=${name#*:}; export ZT_LIB=$R/zlib.ts_amd/build/${spec#*=}/libzt.so
  ps="$ch,128,1,128,8,16,16,1"
  timeout -k 10 300 python tools/ratio_gate.py "$ps" > gpurun_out/r04s3/gate_$name.log 2>&1
  ZT_DF_PARAMS=$ps timeout -k 10 300 python bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-api > gpurun_out/r04s3/bench_$name.log 2>&1
  echo "[$name] $(grep '\[' gpurun_out/r04s3/gate_$name.log | sed 's/.*\] //' | cut -c1-170) | bench $(tail -1 gpurun_out/r04s3/bench_$name.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["match_kernel_ms"], d["ratio"])')"
done
