"""HBM traffic per launch from rocprofv3 PMC passes of bench.py (each pass
runs the measured step twice: the correctness step and one timed step).

Read bytes come from the L2's memory-side read requests by size,
    32 x TCC_EA0_RDREQ_32B + 64 x TCC_EA0_RDREQ_64B + 128 x TCC_EA0_RDREQ_128B,
one rule for every kernel.  It is calibrated on known-byte kernels
(tools/micro/pmc_calib.hip, tools/gpu_pmc_calib.sh, profiles/r04_pmc_calib.txt):
16-, 4- and 2-byte-per-lane coalesced reads and 4-byte LDS-DMA of a 1 GiB
buffer all give 1.000 GiB, while FETCH_SIZE gives 0.500 for each of them (it
tallies a 128-byte request as 64 bytes, MI355X_MICROARCH.md's "half of a
streaming read") -- so the old rule of doubling FETCH_SIZE for some kernels
only is replaced.  32 x TCC_EA0_RDREQ_DRAM_32B (the same requests counted in
32-byte units, DRAM-bound only) is reported beside it, and the raw FETCH_SIZE
too.  WRITE_SIZE is exact for coalesced stores (1.000 in the calibration).
Writes profiles/pmc_traffic.json with the sha256 of the kernel sources it was
measured on; bench.py reports roofline.traffic only when its own sources have
that digest (a stale file gives null).

  python tools/pmc_traffic.py OUT.json fetch_dir=FETCH_SIZE req_dir=REQ write_dir=WRITE_SIZE
  (directories of the three passes: --pmc FETCH_SIZE; --pmc TCC_EA0_RDREQ_32B
   TCC_EA0_RDREQ_64B TCC_EA0_RDREQ_128B TCC_EA0_RDREQ_DRAM_32B; --pmc WRITE_SIZE)
"""
import collections
import csv
import glob
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..'))
from bench import source_digest  # noqa: E402


def load(d):
    """{kernel: {counter: total}}, {kernel: dispatch count}"""
    f = glob.glob(d + '/*counter_collection.csv')[0]
    tot = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for r in csv.DictReader(open(f)):
        k = r['Kernel_Name'].replace('(anonymous namespace)', 'anon').split('(')[0].split('::')[-1]
        tot[k][r['Counter_Name']] += float(r['Counter_Value'])
        disp[k].add(r['Dispatch_Id'])
    return tot, {k: len(v) for k, v in disp.items()}


def main():
    out_path, fetch_dir, req_dir, write_dir = sys.argv[1:5]
    fetch, fd = load(fetch_dir)
    req, rd = load(req_dir)
    write, wd = load(write_dir)
    out = {}
    for k in sorted(set(fetch) | set(req) | set(write)):
        nf, nr, nw = max(1, fd.get(k, 0)), max(1, rd.get(k, 0)), max(1, wd.get(k, 0))
        q = req.get(k, {})
        read = (32 * q.get('TCC_EA0_RDREQ_32B', 0) + 64 * q.get('TCC_EA0_RDREQ_64B', 0) +
                128 * q.get('TCC_EA0_RDREQ_128B', 0)) / nr
        out[k] = {"launches": nr,
                  "read_bytes": read,
                  "read_bytes_dram": 32 * q.get('TCC_EA0_RDREQ_DRAM_32B', 0) / nr,
                  "fetch_size_raw_bytes": fetch.get(k, {}).get('FETCH_SIZE', 0) * 1024 / nf,
                  "write_bytes": write.get(k, {}).get('WRITE_SIZE', 0) * 1024 / nw}
        out[k]["traffic_bytes"] = out[k]["read_bytes"] + out[k]["write_bytes"]
    json.dump({"source": "rocprofv3 PMC passes of bench.py --steps 1 --warmup 0 (1 GiB mixed corpus): "
                         "FETCH_SIZE; TCC_EA0_RDREQ_32B/64B/128B + TCC_EA0_RDREQ_DRAM_32B; WRITE_SIZE",
               "correction": "read bytes = 32 x RDREQ_32B + 64 x RDREQ_64B + 128 x RDREQ_128B for every kernel "
                             "(calibrated: known-byte coalesced / LDS-DMA reads give 1.000 of their bytes, "
                             "FETCH_SIZE 0.500; profiles/r04_pmc_calib.txt); write bytes = WRITE_SIZE",
               "source_sha256": source_digest(),
               "kernels": out}, open(out_path, 'w'), indent=1)
    print(f"{'kernel':24s} {'read GB':>9s} {'(dram)':>9s} {'FETCH_SIZE':>10s} {'write GB':>9s} {'total GB':>9s}")
    for k, v in out.items():
        print(f"{k:24s} {v['read_bytes']/1e9:9.3f} {v['read_bytes_dram']/1e9:9.3f} "
              f"{v['fetch_size_raw_bytes']/1e9:10.3f} {v['write_bytes']/1e9:9.3f} {v['traffic_bytes']/1e9:9.3f}")


if __name__ == "__main__":
    main()
