# Deflate throughput per generator and level: match_kernel and whole-pipeline
# kernel time (HIP events inside libzt), ratio vs the reference's ratio on the
# same generator (1 MiB windows, measured with the oracle: see REF).
import os, sys, time; sys.path.insert(0, 'zlib.ts_amd/py')
import torch, ztamd
REF = {'wordsalad': 0.15455, 'xorshift32': 1.00075, 'structured': 0.4898}
n = int(os.environ.get('SIZE', 256 << 20))
d = torch.empty(n, dtype=torch.uint8, device='cuda')
c = torch.empty(ztamd.deflate_bound(n), dtype=torch.uint8, device='cuda')
o = torch.empty(n + 4096, dtype=torch.uint8, device='cuda')
ip = ztamd.InflatePlan(c.numel(), n)
for level in [int(x) for x in os.environ.get('LEVELS', '6,1').split(',')]:
    p = ztamd.DeflatePlan(n, level=level)
    for kind in ['wordsalad', 'xorshift32', 'structured']:
        ztamd.synth_dev(kind, 3, d.data_ptr(), n)
        clen = p.run(d.data_ptr(), n, c.data_ptr())
        olen, _ = ip.run(c.data_ptr(), clen, o.data_ptr(), o.numel())
        ok = olen == n and torch.equal(o[:n], d)
        ztamd.timing_enable(True)
        t0 = time.time(); clen = p.run(d.data_ptr(), n, c.data_ptr()); dt = time.time() - t0
        olen, _ = ip.run(c.data_ptr(), clen, o.data_ptr(), o.numel())
        t = ztamd.timing_read(); ztamd.timing_enable(False)
        g = n / 2**30
        print(f"L{level} {kind:10s} ok={ok} ratio {clen / n:.4f} vs_ref {clen / n / REF[kind]:.4f} | "
              f"match {g / (t['deflate_ms'] * 1e-3):.2f} GiB/s pipeline {g / (t['deflate_pipeline_ms'] * 1e-3):.2f} "
              f"GiB/s api {g / dt:.2f} GiB/s | inflate {g / (t['inflate_ms'] * 1e-3):.2f} GiB/s", flush=True)
    p.close()
