#!/bin/bash
# Per-generator kernel stats (256 MiB each) for two libraries: in-tree and $2 (build/exp_NAME)
#   usage: tools/gpu_kindab.sh TAG NAME [kernel-regex [NAME2]]
set -e
TAG=$1; V=$2; KRE=${3:-expand|copy|tokenize}
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for k in wordsalad xorshift32 structured; do
  for L in in-tree $V $4; do
    if [ "$L" = in-tree ]; then LIB=""; else LIB=$R/zlib.ts_amd/build/exp_$L/libzt.so; fi
    cd /tmp
    ZT_LIB=$LIB timeout -k 10 240 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/${TAG}_${k}_$L -o run -- python3 $R/tools/kind_time.py 256 $k > $R/gpurun_out/${TAG}_${k}_$L.log 2>&1
    cd $R
    echo "== $k [$L] $(python3 -c "
import csv, re
out = []
for r in csv.DictReader(open('gpurun_out/${TAG}_${k}_$L/run_kernel_stats.csv')):
    n = re.split(r'[(<]', r['Name'].replace('zt::(anonymous namespace)::', ''))[0]
    if re.search(r'$KRE', n): out.append(f'{n} {float(r[\"AverageNs\"])/1e6:.3f}')
print('  '.join(out))
")"
  done
done
