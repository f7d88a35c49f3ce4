#!/bin/bash
# optparse group of 16 positions per lane (fewer VGPRs, more waves) vs 32: kernel time + L2 reads
set -e
R=$GRAFT_REPO_ROOT; mkdir -p gpurun_out/r04g16
export TMPDIR=/tmp
for spec in base= g16=sw_g16 g16p2=sw_g16p2 base2= g16b=sw_g16 g16p2b=sw_g16p2; do
  name=${spec%%=*}; v=${spec#*=}
  if [ -n "$v" ]; then export ZT_LIB=$R/zlib.ts_amd/build/$v/libzt.so; else unset ZT_LIB; fi
  cd /tmp
  timeout -s KILL 180 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/r04g16/prof_$name -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-api > $R/gpurun_out/r04g16/prof_$name.log 2>&1
  cd $R
  echo "[$name] $(grep optparse_kernel gpurun_out/r04g16/prof_$name/run_kernel_stats.csv | cut -d, -f2-4) ratio $(grep -o '"ratio": [0-9.]*' gpurun_out/r04g16/prof_$name.log | head -1)"
done
for spec in g16=sw_g16 g16p2=sw_g16p2; do
  name=${spec%%=*}; export ZT_LIB=$R/zlib.ts_amd/build/${spec#*=}/libzt.so
  cd /tmp
  timeout -s KILL 180 rocprofv3 --pmc TCC_EA0_RDREQ_32B TCC_EA0_RDREQ_64B TCC_EA0_RDREQ_128B TCC_EA0_RDREQ_DRAM_32B -f csv -d $R/gpurun_out/r04g16/pmcq_$name -o run -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-api > $R/gpurun_out/r04g16/pmcq_$name.log 2>&1
  cd $R
done
