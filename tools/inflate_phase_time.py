# Two-phase inflate: per-corpus timing of phase A (tokenize) and the whole
# inflate pipeline, device-resident (256 MiB per corpus).
import os, sys, time; sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', 'zlib.ts_amd', 'py'))
import torch, ztamd as zt
n = 256 << 20
kinds = sys.argv[1].split(",") if len(sys.argv) > 1 else ["wordsalad", "structured", "xorshift32", "mixed"]
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 3
for kind in kinds:
    d_in = torch.empty(n, dtype=torch.uint8, device="cuda")
    zt.synth_dev(kind, 5, d_in.data_ptr(), n)
    bound = zt.deflate_bound(n)
    d_c = torch.empty(bound, dtype=torch.uint8, device="cuda")
    d_o = torch.empty(n + 4096, dtype=torch.uint8, device="cuda")
    dp = zt.DeflatePlan(n); ip = zt.InflatePlan(bound, n)
    clen = dp.run(d_in.data_ptr(), n, d_c.data_ptr())
    ip.run(d_c.data_ptr(), clen, d_o.data_ptr(), d_o.numel())
    torch.cuda.synchronize()
    assert torch.equal(d_o[:n], d_in)
    zt.timing_enable(True)
    for _ in range(iters):
        dp.run(d_in.data_ptr(), n, d_c.data_ptr())
        ip.run(d_c.data_ptr(), clen, d_o.data_ptr(), d_o.numel())
    torch.cuda.synchronize()
    t = zt.timing_read(); zt.timing_enable(False)
    f = lambda a, b: t[a] / max(1, t[b])
    print(f"{kind:11s} ratio {clen/n:.4f} match {f('deflate_ms','deflate_launches'):7.2f} ms  deflate {f('deflate_pipeline_ms','deflate_pipelines'):7.2f} ms  "
          f"tokenize {f('inflate_tok_ms','inflate_toks'):7.2f} ms  inflate {f('inflate_ms','inflate_launches'):7.2f} ms", flush=True)
    dp.close(); ip.close()
    del d_in, d_c, d_o
