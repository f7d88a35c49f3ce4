#!/bin/bash
# Checksum kernel segment-shape variants: the checksum tests and rocprofv3
# kernel stats of checksum_segments per variant (1 GiB device-resident).
#   usage: tools/gpu_ck_var.sh TAG VARIANT...   ("" = in-tree libzt.so)
set -e
TAG=$1; shift
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in "$@"; do
  if [ "$v" = "-" ]; then L=""; else L=$R/zlib.ts_amd/build/exp_$v/libzt.so; fi
  ZT_LIB=$L timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_checksums.py \
    > gpurun_out/${TAG}_${v}_pytest.log 2>&1 || { tail -20 gpurun_out/${TAG}_${v}_pytest.log; exit 1; }
  cd /tmp
  ZT_LIB=$L timeout -k 10 180 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/${TAG}_${v}_prof -o run -- python3 $R/tools/ck_time.py > $R/gpurun_out/${TAG}_${v}_prof.log 2>&1
  cd $R
  echo "[$v] $(tail -n 1 gpurun_out/${TAG}_${v}_pytest.log) $(grep checksums gpurun_out/${TAG}_${v}_prof.log) kernel $(python3 -c "
import csv
for r in csv.DictReader(open('gpurun_out/${TAG}_${v}_prof/run_kernel_stats.csv')):
    if 'checksum_segments' in r['Name']: print(r['AverageNs'])
")"
done
