#!/bin/bash
# FETCH_SIZE / WRITE_SIZE and the read-request-size counters on known-byte
# kernels (tools/micro/pmc_calib.hip): which counter gives the bytes read
set -e
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out/calib
cd /tmp
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE -f csv -d $R/gpurun_out/calib/f -o run -- $R/tools/micro/pmc_calib > $R/gpurun_out/calib/f.log 2>&1
timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE -f csv -d $R/gpurun_out/calib/w -o run -- $R/tools/micro/pmc_calib > $R/gpurun_out/calib/w.log 2>&1
timeout -s KILL 60 rocprofv3 --pmc TCC_EA0_RDREQ_32B TCC_EA0_RDREQ_64B TCC_EA0_RDREQ_128B TCC_EA0_RDREQ_DRAM_32B -f csv -d $R/gpurun_out/calib/q -o run -- $R/tools/micro/pmc_calib > $R/gpurun_out/calib/q.log 2>&1
cd $R
python3 - <<'PY'
import csv, glob, collections
vals = collections.defaultdict(float)
names = {}
for d in ("f", "w", "q"):
    f = glob.glob(f"gpurun_out/calib/{d}/*counter_collection.csv")[0]
    for r in csv.DictReader(open(f)):
        vals[(d, int(r["Dispatch_Id"]), r["Counter_Name"])] += float(r["Counter_Value"])
        names[(d, int(r["Dispatch_Id"]))] = r["Kernel_Name"].split("(")[0]
G = 2**30
for disp in range(10, 17):
    k = names.get(("f", disp), "?")
    fetch = vals[("f", disp, "FETCH_SIZE")] * 1024 / G
    write = vals[("w", disp, "WRITE_SIZE")] * 1024 / G
    q = lambda c: vals[("q", disp, c)]
    req = (32 * q("TCC_EA0_RDREQ_32B") + 64 * q("TCC_EA0_RDREQ_64B") + 128 * q("TCC_EA0_RDREQ_128B")) / G
    dram = 32 * q("TCC_EA0_RDREQ_DRAM_32B") / G
    print(f"{k:16s} FETCH_SIZE {fetch:6.3f}  32/64/128B requests {req:6.3f}  DRAM_32B x 32 {dram:6.3f}  WRITE_SIZE {write:6.3f}  (x 1 GiB)")
PY
