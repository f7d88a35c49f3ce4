# SIMT tokenizer phase cycles (libzt built with -DZT_TK_TIME, ZT_LIB=...): per
# round of 64 x 480 bits, staging / pass 1 / repairs / pass 2, on 256 MiB of
# one generator deflated by this engine (tokenize_kernel's units).
#   usage: python tools/tk_time.py [MiB] [generator...]
import ctypes, os, sys
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
buf = (ctypes.c_ulonglong * 8)()
for kind in sys.argv[2:] or ["wordsalad", "structured", "mixed"]:
    zt.synth_dev(kind, 11, d_in.data_ptr(), n)
    clen = dp.run(d_in.data_ptr(), n, d_c.data_ptr())
    ip.run(d_c.data_ptr(), clen, d_out.data_ptr(), d_out.numel())
    torch.cuda.synchronize()
    zt.lib.zt_debug_tk_time(buf)
    ip.run(d_c.data_ptr(), clen, d_out.data_ptr(), d_out.numel())
    torch.cuda.synchronize()
    zt.lib.zt_debug_tk_time(buf)
    assert torch.equal(d_out[:n], d_in[:n])
    r = max(1, buf[4])
    print(f"{kind:10s} {buf[4]} rounds, {buf[5] / r:.2f} repair iterations per round; cycles per round: "
          f"stage {buf[0] / r:.0f} (store wait {buf[7] / r:.0f})  pass1 {buf[1] / r:.0f}  repairs {buf[2] / r:.0f}  pass2 {buf[3] / r:.0f}", flush=True)
