#!/bin/bash
# A/B of library builds on one box: optional GPU tests on the main build, then
# per library the 16-window ratio gate and the 1 GiB bench's kernel times.
#   usage: TAG=r05a TESTS="tests/test_gpu_deflate.py ..." tools/gpu_libab.sh main build/r05_x ...
# ("main" = zlib.ts_amd/libzt.so; others are zlib.ts_amd/<dir>/libzt.so,
# built by VAR_PREFIX=r05_ tools/build_variant.sh)
set -e
O=gpurun_out/${TAG:-ab}; mkdir -p $O
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread $TESTS > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
  tail -1 $O/pytest.log
fi
i=0
for L in "$@"; do
  i=$((i+1))
  if [ "$L" = main ]; then unset ZT_LIB; else export ZT_LIB=$PWD/zlib.ts_amd/$L/libzt.so; fi
  n=$(echo $L | tr / _)_$i
  if [ -z "$NOGATE" ]; then
    timeout -k 10 300 python tools/ratio_gate.py "${PARAMS:-}" > $O/gate_$n.log 2>&1
  fi
  timeout -k 10 300 python bench.py --steps ${STEPS:-5} --warmup 2 --no-cpu-baseline --no-api --no-per-generator > $O/bench_$n.log 2>&1
  echo "$L | $(grep -o 'worst.*' $O/gate_$n.log 2>/dev/null) | $(tail -1 $O/bench_$n.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("bench", d["value"], "ratio", d["ratio"], "deflate", d["deflate_pipeline_ms"], "match", d["match_kernel_ms"], "inflate", d["inflate_kernel_ms"])')"
done
