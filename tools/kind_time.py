# Per-generator cost of the bench pipeline: 256 MiB of one generator (device
# synthetic corpus) deflated and inflated through the device plans,
# kernel intervals from the library's HIP-event timers (ms per 256 MiB), and the
# ratio.   usage: python tools/kind_time.py [MiB] [generator...]
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, '..', 'zlib.ts_amd', 'py'))
import torch  # noqa: E402
import ztamd as zt  # noqa: E402

n = (int(sys.argv[1]) if len(sys.argv) > 1 else 256) << 20
d_in = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
d_c = torch.empty(zt.deflate_bound(n) + 64, dtype=torch.uint8, device="cuda")
d_out = torch.empty(n + 4096, dtype=torch.uint8, device="cuda")
dp = zt.DeflatePlan(n, level=6)
ip = zt.InflatePlan(zt.deflate_bound(n) + 64, n)
for kind in sys.argv[2:] or ["wordsalad", "xorshift32", "structured"]:
    zt.synth_dev(kind, 11, d_in.data_ptr(), n)
    clen = dp.run(d_in.data_ptr(), n, d_c.data_ptr())
    ip.run(d_c.data_ptr(), clen, d_out.data_ptr(), d_out.numel())
    torch.cuda.synchronize()
    zt.timing_enable(True)
    for _ in range(3):
        clen = dp.run(d_in.data_ptr(), n, d_c.data_ptr())
        olen, _ = ip.run(d_c.data_ptr(), clen, d_out.data_ptr(), d_out.numel())
    torch.cuda.synchronize()
    t = zt.timing_read()
    zt.timing_enable(False)
    assert olen == n and torch.equal(d_out[:n], d_in[:n])
    k = lambda a, b: t[a] / max(1, t[b])
    print(f"{kind:10s} ratio {clen / n:.4f}  match {k('deflate_ms', 'deflate_launches'):7.2f}  "
          f"deflate {k('deflate_pipeline_ms', 'deflate_pipelines'):7.2f}  inflate {k('inflate_ms', 'inflate_launches'):7.2f}  "
          f"tokenize {k('inflate_tok_ms', 'inflate_toks'):6.2f} ms per {n >> 20} MiB", flush=True)
