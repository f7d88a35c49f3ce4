#!/bin/bash
# encode_kernel token cache 32 / 48 / 64 per thread: bench time (streams identical)
set -e
R=$GRAFT_REPO_ROOT; mkdir -p gpurun_out/r04ec2
for spec in ec32=sw_ec32 ec48=sw_ec48 ec64=sw_ec64 ec32b=sw_ec32 ec48b=sw_ec48 ec64b=sw_ec64; do
  name=${spec%%=*}; export ZT_LIB=$R/zlib.ts_amd/build/${spec#*=}/libzt.so
  cd /tmp
  timeout -s KILL 180 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/r04ec2/prof_$name -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-api > $R/gpurun_out/r04ec2/prof_$name.log 2>&1
  cd $R
  echo "[$name] $(grep encode_kernel gpurun_out/r04ec2/prof_$name/run_kernel_stats.csv | cut -d, -f2-4) $(tail -1 gpurun_out/r04ec2/prof_$name.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["deflate_pipeline_ms"])')"
done
