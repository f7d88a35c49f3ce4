#!/bin/bash
# A/B of libzt variants (build/<prefix><name>/libzt.so, tools/build_variant.sh) on
# the bench workload: bench line + rocprofv3 kernel stats of the deflate post-match kernels.
#   usage: tools/gpu_pkvar.sh PREFIX NAME... ("default" = the in-tree libzt.so)
set -e
R=$GRAFT_REPO_ROOT
P=$1; shift
mkdir -p $R/gpurun_out
export TMPDIR=/tmp
cd /tmp
for v in "$@"; do
  if [ $v = default ]; then unset ZT_LIB; else export ZT_LIB=$R/zlib.ts_amd/build/$P$v/libzt.so; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/$P$v -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-api > $R/gpurun_out/$P$v.log 2>&1
  echo "== $v"; grep "^{" $R/gpurun_out/$P$v.log | python3 -c "import sys,json; [print(d['value'], d['deflate_pipeline_ms'], d['ratio'], d['inflate_kernel_ms']) for d in map(json.loads, sys.stdin)]"
  grep -E "parse_kernel|block_kernel|price_kernel|optparse_kernel|encode_kernel|tokenize_kernel" $R/gpurun_out/$P$v/run_kernel_stats.csv | cut -d, -f1-4 | sed 's/zt::(anonymous namespace):://; s/(zt::DeflateParams)//'
done
