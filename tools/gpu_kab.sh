#!/bin/bash
# rocprofv3 kernel stats of the 1 GiB bench for several libzt builds
# (ZT_LIB): usage tools/gpu_kab.sh TAG name=path ...   ("new" = in-tree)
set -e
TAG=$1; shift
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
for spec in "$@"; do
  name=${spec%%=*}; lib=${spec#*=}
  if [ "$lib" = new ]; then unset ZT_LIB; else export ZT_LIB=$R/$lib; fi
  cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/$TAG/$name -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-api > $R/gpurun_out/$TAG/$name.log 2>&1
  cd $R
  echo "== $name $(tail -1 gpurun_out/$TAG/$name.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["deflate_pipeline_ms"], d["inflate_kernel_ms"])')"
  cut -d, -f1,3,4 gpurun_out/$TAG/$name/run_kernel_stats.csv | sed 's/zt::(anonymous namespace):://; s/(.*)"/"/' | head -16
done
