# copy_kernel phase cycles (build with -DZT_CP_TIME, load with ZT_LIB): the
# bench's 1 GiB mixed corpus, deflated once, inflated twice (the second
# counted).  Phases per step: DMA issue + descriptor wait, descriptor + ring
# reads, ring writes (+ in-step resolution), output flush.
import ctypes, os, sys
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, '..', 'zlib.ts_amd', 'py'))
import torch  # noqa: E402
import ztamd as zt  # noqa: E402
n = (int(sys.argv[1]) if len(sys.argv) > 1 else 1024) << 20
kind = sys.argv[2] if len(sys.argv) > 2 else "mixed"
d_in = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
d_c = torch.empty(zt.deflate_bound(n) + 64, dtype=torch.uint8, device="cuda")
d_out = torch.empty(n + 4096, dtype=torch.uint8, device="cuda")
zt.synth_dev(kind, 11, d_in.data_ptr(), n)
clen = zt.DeflatePlan(n, level=6).run(d_in.data_ptr(), n, d_c.data_ptr())
ip = zt.InflatePlan(zt.deflate_bound(n) + 64, n)
ip.run(d_c.data_ptr(), clen, d_out.data_ptr(), d_out.numel())
torch.cuda.synchronize()
lib = zt.lib
buf = (ctypes.c_ulonglong * 8)()
lib.zt_debug_cp_time(buf)
ip.run(d_c.data_ptr(), clen, d_out.data_ptr(), d_out.numel())
torch.cuda.synchronize()
lib.zt_debug_cp_time(buf)
assert torch.equal(d_out[:n], d_in[:n])
steps, waves = buf[6], buf[7]
names = ["dma+wait", "reads", "writes", "flush"]
tot = sum(buf[k] for k in range(4))
print(f"{kind} {n >> 20} MiB: {waves} waves, {steps} steps, {tot / max(1, steps):.0f} cycles per step: " +
      ", ".join(f"{names[k]} {buf[k] / max(1, steps):.0f}" for k in range(4)), flush=True)
