#!/bin/bash
# copy_kernel phase cycles (ZT_CP_TIME build) + the bench's kernel stats at HEAD
set -e
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for k in mixed wordsalad; do
  ZT_LIB=$R/zlib.ts_amd/build/exp_cptime/libzt.so timeout -k 10 200 python tools/cp_time.py 1024 $k 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/${1}_cptime.log
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/${1}_bprof -o run -- python3 $R/bench.py --no-cpu-baseline --no-api --steps 5 > $R/gpurun_out/${1}_bprof.log 2>&1
cd $R
tail -n 1 gpurun_out/${1}_bprof.log
python3 -c "
import csv, re
for r in csv.DictReader(open('gpurun_out/${1}_bprof/run_kernel_stats.csv')):
    n = re.split(r'[(<]', r['Name'].replace('zt::(anonymous namespace)::', ''))[0][:28]
    print(f'  {n:28s} {int(r[\"Calls\"]):4d} {float(r[\"AverageNs\"])/1e6:8.3f} ms')
"
