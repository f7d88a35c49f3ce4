"""HBM traffic per launch from two rocprofv3 PMC passes of bench.py
(--pmc FETCH_SIZE, --pmc WRITE_SIZE; each pass runs the measured step twice:
the correctness step and one timed step).  FETCH_SIZE/WRITE_SIZE are in KB.
Per MI355X_MICROARCH.md (HBM/rocprofv3): on gfx950 FETCH_SIZE reports half of
the bytes of a streaming read, so fetch bytes are doubled; WRITE_SIZE is
taken as is.  Writes profiles/pmc_traffic.json, which bench.py uses for
roofline.traffic.

  python tools/pmc_traffic.py gpurun_out/pmcf gpurun_out/pmcw profiles/pmc_traffic.json
"""
import collections
import csv
import glob
import json
import sys


def load(d, name):
    f = glob.glob(d + '/*counter_collection.csv')[0]
    tot = collections.defaultdict(float)
    disp = collections.defaultdict(set)
    for r in csv.DictReader(open(f)):
        if r['Counter_Name'] != name:
            continue
        k = r['Kernel_Name'].replace('(anonymous namespace)', 'anon').split('(')[0].split('::')[-1]
        tot[k] += float(r['Counter_Value'])
        disp[k].add(r['Dispatch_Id'])
    return tot, disp


fetch, fd = load(sys.argv[1], 'FETCH_SIZE')
write, wd = load(sys.argv[2], 'WRITE_SIZE')
out = {}
for k in sorted(set(fetch) | set(write)):
    n = max(1, len(fd.get(k, ())))
    m = max(1, len(wd.get(k, ())))
    out[k] = {"launches": n, "fetch_bytes_raw": fetch.get(k, 0) * 1024 / n,
              "fetch_bytes": 2 * fetch.get(k, 0) * 1024 / n, "write_bytes": write.get(k, 0) * 1024 / m}
    out[k]["traffic_bytes"] = out[k]["fetch_bytes"] + out[k]["write_bytes"]
json.dump({"source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE of bench.py --steps 1 --warmup 0 (1 GiB mixed corpus)",
           "correction": "fetch doubled (gfx950 FETCH_SIZE = half of streamed bytes, MI355X_MICROARCH.md)",
           "kernels": out}, open(sys.argv[3], 'w'), indent=1)
for k, v in out.items():
    print(f"{k:24s} fetch {v['fetch_bytes']/1e9:8.3f} GB  write {v['write_bytes']/1e9:8.3f} GB per launch")
