# Host stage timestamps of one device-resident 1 GiB inflate (the bench
# corpus, or one generator), ZT_INF_TIMING=1 set by the caller:
#   python tools/inf_timing.py [kind]
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', 'zlib.ts_amd', 'py'))
import torch, ztamd as zt
n = 1 << 30
d_in = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
zt.synth_dev(sys.argv[1] if len(sys.argv) > 1 else "mixed", 1, d_in.data_ptr(), n)
d_c = torch.empty(zt.deflate_bound(n) + 64, dtype=torch.uint8, device="cuda")
clen = zt.DeflatePlan(n, level=6).run(d_in.data_ptr(), n, d_c.data_ptr())
d_out = torch.empty(n + 4096, dtype=torch.uint8, device="cuda")
ip = zt.InflatePlan(zt.deflate_bound(n) + 64, n)
for k in range(3):
    print(f"-- call {k}", file=sys.stderr, flush=True)
    ip.run(d_c.data_ptr(), clen, d_out.data_ptr(), d_out.numel())
torch.cuda.synchronize()
