#!/bin/bash
# encode_kernel tokens kept in registers per thread (ZT_ENC_NCACHE 16 / 24 / 32):
# bench time (streams identical) and the kernel's L2 read requests
set -e
R=$GRAFT_REPO_ROOT; mkdir -p gpurun_out/r04ec
export TMPDIR=/tmp
for spec in base= ec24=sw_ec24 ec32=sw_ec32 base2= ec32b=sw_ec32; do
  name=${spec%%=*}; v=${spec#*=}
  if [ -n "$v" ]; then export ZT_LIB=$R/zlib.ts_amd/build/$v/libzt.so; else unset ZT_LIB; fi
  timeout -k 10 300 python bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-api > gpurun_out/r04ec/bench_$name.log 2>&1
  echo "[$name] bench $(tail -1 gpurun_out/r04ec/bench_$name.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["deflate_pipeline_ms"], d["match_kernel_ms"], d["ratio"])')"
done
for spec in base= ec32=sw_ec32; do
  name=${spec%%=*}; v=${spec#*=}
  if [ -n "$v" ]; then export ZT_LIB=$R/zlib.ts_amd/build/$v/libzt.so; else unset ZT_LIB; fi
  cd /tmp
  timeout -s KILL 180 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/r04ec/prof_$name -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-api > $R/gpurun_out/r04ec/prof_$name.log 2>&1
  timeout -s KILL 180 rocprofv3 --pmc TCC_EA0_RDREQ_32B TCC_EA0_RDREQ_64B TCC_EA0_RDREQ_128B TCC_EA0_RDREQ_DRAM_32B -f csv -d $R/gpurun_out/r04ec/pmcq_$name -o run -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-api > $R/gpurun_out/r04ec/pmcq_$name.log 2>&1
  cd $R
  grep encode_kernel gpurun_out/r04ec/prof_$name/run_kernel_stats.csv | cut -d, -f2-4
done
