# Per-kernel SQ counter summary of a rocprofv3 --pmc run (counter_collection.csv):
# wave-cycle split into parked (s_waitcnt / barrier), issue-stalled and issuing
import csv, collections, re, sys
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for r in csv.DictReader(open(sys.argv[1])):
    m = re.search(r'::(\w+)(<[^(]*>)?\(', r['Kernel_Name'])
    k = m.group(1) if m else r['Kernel_Name'][:30]
    agg[k][r['Counter_Name']] += float(r['Counter_Value'])
for k, v in sorted(agg.items(), key=lambda kv: -kv[1]['SQ_WAVE_CYCLES']):
    w = v['SQ_WAVE_CYCLES'] or 1
    if w < 1e8: continue
    print(f"{k:20s} wave_cyc {w:9.3g}  parked {v['SQ_WAIT_ANY']/w:.2f}  issue-stall {v['SQ_WAIT_INST_ANY']/w:.2f}"
          f" (lds {v['SQ_WAIT_INST_LDS']/w:.2f})  issuing {v['SQ_ACTIVE_INST_ANY']/w:.2f} (valu {v['SQ_ACTIVE_INST_VALU']/w:.2f})"
          f"  valu/lds instr {v['SQ_INSTS_VALU']:.3g}/{v['SQ_INSTS_LDS']:.3g}")
