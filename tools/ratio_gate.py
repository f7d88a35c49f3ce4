# Ratio gate table: this build's level-6 bytes over the
# reference's whole-window bytes on the 16 windows of tests/ratio_corpus.py,
# per window and per generator, plus match-kernel / pipeline time per
# generator.  Each argument is a ZT_DF_PARAMS set to compare ("" = level 6).
#   usage: python tools/ratio_gate.py ["" "32,128,1,128,4,16,16,1" ...]
import os, sys
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, '..', 'tests')); sys.path.insert(0, os.path.join(HERE, '..', 'zlib.ts_amd', 'py'))
import torch, ztamd as zt, zt_oracle
from ratio_corpus import windows, reference_sizes, GENERATORS
o = zt_oracle.Oracle()
wins = windows(o)
refs = reference_sizes(o, wins)
n = max(len(w[2]) for w in wins)
d_in = torch.empty(n, dtype=torch.uint8, device="cuda")
d_c = torch.empty(zt.deflate_bound(n), dtype=torch.uint8, device="cuda")
dp = zt.DeflatePlan(n, level=6)
for ps in (sys.argv[1:] or [""]):
    if ps:
        os.environ["ZT_DF_PARAMS"] = ps
    else:
        os.environ.pop("ZT_DF_PARAMS", None)
    agg = {g: [0, 0, 0.0, 0.0] for g in GENERATORS}
    worst = (0, "")
    for (g, label, data), ref in zip(wins, refs):
        d_in[:len(data)] = torch.frombuffer(bytearray(data), dtype=torch.uint8).cuda()
        dp.run(d_in.data_ptr(), len(data), d_c.data_ptr())
        zt.timing_enable(True)
        clen = dp.run(d_in.data_ptr(), len(data), d_c.data_ptr())
        torch.cuda.synchronize()
        t = zt.timing_read(); zt.timing_enable(False)
        a = agg[g]; a[0] += clen; a[1] += ref; a[2] += t['deflate_ms']; a[3] += t['deflate_pipeline_ms']
        worst = max(worst, (clen / ref, label))
    row = "  ".join(f"{g} {a[0]/a[1]:.4f} ({a[2]:.2f}/{a[3]:.2f} ms)" for g, a in agg.items())
    print(f"[{ps or 'level6'}] {row}  worst {worst[1]} {worst[0]:.4f}", flush=True)
