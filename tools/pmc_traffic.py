"""HBM traffic per launch from two rocprofv3 PMC passes of bench.py
(--pmc FETCH_SIZE, --pmc WRITE_SIZE; each pass runs the measured step twice:
the correctness step and one timed step).  FETCH_SIZE/WRITE_SIZE are in KB.
Per MI355X_MICROARCH.md (HBM/rocprofv3): on gfx950 FETCH_SIZE reports half of
the bytes of a wide coalesced streaming read, so fetch bytes are doubled for
the kernels whose reads are such streams (STREAMING below: the match kernel's
input/history loads, the checksum, sync scan and gather passes); the other
kernels' reads (gathers, pointer chases, LDS-DMA of scattered slices) are an
uncalibrated access pattern for that correction, so their raw FETCH_SIZE is
kept and flagged.  WRITE_SIZE is taken as is.  Writes
profiles/pmc_traffic.json with the sha256 of the kernel sources it was
measured on; bench.py reports roofline.traffic only when its own sources have
that digest (a stale file gives null).

  python tools/pmc_traffic.py gpurun_out/pmcf gpurun_out/pmcw profiles/pmc_traffic.json
"""
import collections
import csv
import glob
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..'))
from bench import source_digest  # noqa: E402

# kernels whose global reads are wide coalesced streams (the guide's calibrated case)
STREAMING = {"match_kernel", "checksum_segments", "find_syncs", "gather_blocks", "synth_kernel"}


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
    f = 2 if k in STREAMING else 1
    out[k] = {"launches": n, "fetch_bytes_raw": fetch.get(k, 0) * 1024 / n,
              "fetch_bytes": f * fetch.get(k, 0) * 1024 / n, "write_bytes": write.get(k, 0) * 1024 / m,
              "fetch_correction": "x2 (streaming read)" if f == 2 else "none (uncalibrated access pattern)"}
    out[k]["traffic_bytes"] = out[k]["fetch_bytes"] + out[k]["write_bytes"]
json.dump({"source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE of bench.py --steps 1 --warmup 0 (1 GiB mixed corpus)",
           "correction": "fetch doubled for wide coalesced streaming readers only (gfx950 FETCH_SIZE = half of "
                         "streamed bytes, MI355X_MICROARCH.md HBM section); other kernels raw",
           "source_sha256": source_digest(),
           "kernels": out}, open(sys.argv[3], 'w'), indent=1)
for k, v in out.items():
    print(f"{k:24s} fetch {v['fetch_bytes']/1e9:8.3f} GB  write {v['write_bytes']/1e9:8.3f} GB per launch")
