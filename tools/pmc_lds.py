"""LDS-array roofline of the match kernel: the fraction
of its CU-cycles in which the LDS array is busy, from one rocprofv3 --pmc
pass of bench.py (SQ_LDS_IDX_ACTIVE = all LDS-array cycles, summed over the
CUs; SQ_LDS_BANK_CONFLICT = the extra cycles bank conflicts cost;
MI355X_MICROARCH.md section LDS) and the kernel's average duration from the
kernel-stats CSV of the same workload:

    busy_frac = LDS_IDX_ACTIVE per launch / (CUs x 2.4 GHz x duration)

and, when the pass also holds them, the SIMDs' VALU time and the waves'
parked share (SQ_INSTS_VALU: wave64 VALU instructions, each 2 cycles of a
SIMD-32's issue -- MI355X_MICROARCH.md; SQ_WAIT_ANY / SQ_WAVE_CYCLES, both in
the same quad-cycle unit):

    valu_busy_frac = 2 x INSTS_VALU per launch / (4 SIMDs x CUs x 2.4 GHz x duration)

Writes profiles/pmc_lds.json with the sha256 of the kernel sources
(bench.source_digest); bench.py reports roofline.lds only when its own
sources carry that digest.

  python tools/pmc_lds.py OUT.json SQ_DIR KERNEL_STATS.csv [kernel]
"""
import collections
import csv
import glob
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..'))
from bench import source_digest  # noqa: E402

CLOCK_HZ = 2.4e9  # MI355X peak engine clock (MI355X_MICROARCH.md)
NUM_CU = 256


def short(name):
    return name.replace('(anonymous namespace)', 'anon').split('(')[0].split('<')[0].split('::')[-1]


def main():
    out_path, sq_dir, stats_csv = sys.argv[1:4]
    kernel = sys.argv[4] if len(sys.argv) > 4 else "match_kernel"
    f = glob.glob(sq_dir + '/*counter_collection.csv')[0]
    tot = collections.defaultdict(float)
    disp = set()
    for r in csv.DictReader(open(f)):
        if short(r['Kernel_Name']) != kernel:
            continue
        tot[r['Counter_Name']] += float(r['Counter_Value'])
        disp.add(r['Dispatch_Id'])
    n = max(1, len(disp))
    avg_ns = None
    for r in csv.DictReader(open(stats_csv)):
        if short(r['Name']) == kernel:
            avg_ns = float(r['AverageNs'])
    if avg_ns is None:
        raise SystemExit(f"{kernel} not in {stats_csv}")
    cu_cycles = NUM_CU * CLOCK_HZ * avg_ns * 1e-9
    active = tot['SQ_LDS_IDX_ACTIVE'] / n
    conflict = tot['SQ_LDS_BANK_CONFLICT'] / n
    valu = tot['SQ_INSTS_VALU'] / n if 'SQ_INSTS_VALU' in tot else None
    res = {"kernel": kernel, "launches": n, "avg_ms": round(avg_ns * 1e-6, 4),
           "valu_busy_frac": round(2 * valu / (4 * cu_cycles), 4) if valu is not None else None,
           "wave_parked_frac": round(tot['SQ_WAIT_ANY'] / tot['SQ_WAVE_CYCLES'], 4)
           if 'SQ_WAIT_ANY' in tot and tot.get('SQ_WAVE_CYCLES') else None,
           "lds_idx_active_per_launch": active, "lds_bank_conflict_per_launch": conflict,
           "busy_frac": round(active / cu_cycles, 4), "bank_conflict_frac": round(conflict / active, 4) if active else None,
           "clock_hz": CLOCK_HZ, "num_cu": NUM_CU, "source_sha256": source_digest(),
           "counters": {k: v / n for k, v in tot.items()}}
    with open(out_path, "w") as fo:
        json.dump(res, fo, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
