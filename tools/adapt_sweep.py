# Per-block search depth sweep (deflate.hip DeflateParams::adapt_depth /
# adapt_thr, ZT_DF_ADAPT="depth,thr"; "" = off): for each setting the
# 16-window ratio gate of tests/ratio_corpus.py (per generator and the worst
# window, this build's level-6 bytes over the reference's) and the match /
# deflate pipeline time per GiB on device-synthetic corpora (the bench's
# mixed corpus, each generator alone, and the source-text sample tiled).
#   usage: python tools/adapt_sweep.py ["" "8,40" "10,20" ...]
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, '..', 'tests'))
sys.path.insert(0, os.path.join(HERE, '..', 'zlib.ts_amd', 'py'))
sys.path.insert(0, os.path.join(HERE, '..'))
import torch  # noqa: E402
import ztamd as zt  # noqa: E402
import zt_oracle  # noqa: E402
from ratio_corpus import windows, reference_sizes, GENERATORS  # noqa: E402
from bench import source_text  # noqa: E402

o = zt_oracle.Oracle()
wins = windows(o)
refs = reference_sizes(o, wins)
n = 1 << 30
d_in = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
d_c = torch.empty(zt.deflate_bound(n) + 64, dtype=torch.uint8, device="cuda")
dp = zt.DeflatePlan(n, level=6)
src = source_text()
corpora = ["mixed", "wordsalad", "structured"] + (["source_text"] if src else [])


def fill(kind):
    if kind == "source_text":
        tile = torch.frombuffer(bytearray(src), dtype=torch.uint8).cuda()
        d_in[:n] = tile.repeat((n + len(src) - 1) // len(src))[:n]
    else:
        zt.synth_dev(kind, 11, d_in.data_ptr(), n)


for ps in (sys.argv[1:] or [""]):
    if ps:
        os.environ["ZT_DF_ADAPT"] = ps
    else:
        os.environ.pop("ZT_DF_ADAPT", None)
    agg = {g: [0, 0] for g in GENERATORS}
    worst = (0, "")
    for (g, label, data), ref in zip(wins, refs):
        d_in[:len(data)] = torch.frombuffer(bytearray(data), dtype=torch.uint8).cuda()
        clen = dp.run(d_in.data_ptr(), len(data), d_c.data_ptr())
        agg[g][0] += clen
        agg[g][1] += ref
        worst = max(worst, (clen / ref, label))
    row = "  ".join(f"{g} {a[0] / a[1]:.4f}" for g, a in agg.items())
    times = []
    for kind in corpora:
        fill(kind)
        dp.run(d_in.data_ptr(), n, d_c.data_ptr())
        torch.cuda.synchronize()
        zt.timing_enable(True)
        for _ in range(2):
            clen = dp.run(d_in.data_ptr(), n, d_c.data_ptr())
        torch.cuda.synchronize()
        t = zt.timing_read()
        zt.timing_enable(False)
        times.append(f"{kind} {t['deflate_ms'] / max(1, t['deflate_launches']):.2f}/"
                     f"{t['deflate_pipeline_ms'] / max(1, t['deflate_pipelines']):.2f} r {clen / n:.4f}")
    print(f"[{ps or 'off'}] gate: {row}  worst {worst[1]} {worst[0]:.4f} | match/pipeline ms per GiB: "
          + "  ".join(times), flush=True)
