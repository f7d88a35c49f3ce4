import os, sys
sys.path.insert(0, 'zlib.ts_amd/py')
import torch, ztamd as zt
n = 1 << 30
for kind in ["mixed", "wordsalad", "xorshift32", "structured"]:
    d_in = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
    zt.synth_dev(kind, 11, d_in.data_ptr(), n)
    d_c = torch.empty(zt.deflate_bound(n) + 64, dtype=torch.uint8, device="cuda")
    clen = zt.DeflatePlan(n, level=6).run(d_in.data_ptr(), n, d_c.data_ptr())
    d_out = torch.empty(n + 4096, dtype=torch.uint8, device="cuda")
    ip = zt.InflatePlan(zt.deflate_bound(n) + 64, n)
    print(kind, clen, flush=True)
    ip.run(d_c.data_ptr(), clen, d_out.data_ptr(), d_out.numel())
    torch.cuda.synchronize()
    del d_in, d_c, d_out, ip
