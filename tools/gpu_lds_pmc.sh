#!/bin/bash
# LDS bank-conflict / activity counters of one bench step (match kernel and the rest).
#   usage: tools/gpu_lds_pmc.sh TAG
TAG=${1:-lds}
R=$GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
cd /tmp
timeout -s KILL 150 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_WAVE_CYCLES -f csv -d $R/gpurun_out/${TAG}_pmc -o run -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-api > $R/gpurun_out/${TAG}.log 2>&1 || { tail -5 $R/gpurun_out/${TAG}.log; exit 1; }
cd $R
python3 - <<PY
import csv, collections
rows = list(csv.DictReader(open("gpurun_out/${TAG}_pmc/run_counter_collection.csv")))
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for r in rows:
    k = r["Kernel_Name"].split("::")[-1].split("(")[0]
    agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, v in sorted(agg.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0))[:8]:
    print(k[:22].ljust(22), " ".join(f"{c.replace('SQ_','')}={v[c]:.3g}" for c in sorted(v)))
PY
