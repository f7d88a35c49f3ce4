#!/bin/bash
# Where the match kernel's cycles go, round 4: two SQ counter passes over one
# bench step (wave-cycle split; LDS activity / conflicts) and the per-wave
# ZT_DF_TIME split per generator (build/var_dftime, -DZT_DF_TIME).
#   usage: tools/gpu_r04_sq.sh TAG
set -e
TAG=${1:-r04sq}
R=$GRAFT_REPO_ROOT; mkdir -p gpurun_out/$TAG; export TMPDIR=/tmp
cd /tmp
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS -f csv -d $R/gpurun_out/$TAG/sq1 -o run -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-api --no-per-generator > $R/gpurun_out/$TAG/sq1.log 2>&1
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_SCA -f csv -d $R/gpurun_out/$TAG/sq2 -o run -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-api --no-per-generator > $R/gpurun_out/$TAG/sq2.log 2>&1
cd $R
python3 tools/sq_summ.py gpurun_out/$TAG/sq1/run_counter_collection.csv > gpurun_out/$TAG/sq1.txt
python3 - > gpurun_out/$TAG/sq2.txt <<PY
import csv, collections, re
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for r in csv.DictReader(open("gpurun_out/$TAG/sq2/run_counter_collection.csv")):
    m = re.search(r'::(\w+)(<[^(]*>)?\(', r['Kernel_Name'])
    k = m.group(1) if m else r['Kernel_Name'][:30]
    agg[k][r['Counter_Name']] += float(r['Counter_Value'])
for k, v in sorted(agg.items(), key=lambda kv: -kv[1]['SQ_WAVE_CYCLES'])[:10]:
    print(k[:22].ljust(22), " ".join(f"{c.replace('SQ_','')}={v[c]:.4g}" for c in sorted(v)))
PY
cat gpurun_out/$TAG/sq1.txt gpurun_out/$TAG/sq2.txt
ZT_LIB=$R/zlib.ts_amd/build/var_dftime/libzt.so timeout -k 10 180 python3 tools/df_time.py wordsalad xorshift32 structured mixed > gpurun_out/$TAG/df_time.log 2>&1
cat gpurun_out/$TAG/df_time.log
