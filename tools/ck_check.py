# C1 checksum kernel: correctness on odd sizes/offsets against zlib, then 1 GiB timing.
import os, sys, time, zlib; sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', 'zlib.ts_amd', 'py'))
import torch, ztamd as zt
n = 1 << 30
d = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
zt.synth_dev("mixed", 3, d.data_ptr(), n)
torch.cuda.synchronize()
host = d[:(64 << 20) + 64].cpu().numpy().tobytes()
for off, m in [(0, 64 << 20), (3, (64 << 20) - 5), (16, 262144 * 3), (5, 1000), (0, 262144 * 8 + 17)]:
    c, a = zt.dev_checksums(d.data_ptr() + off, m)
    b = host[off:off + m]
    assert c == zlib.crc32(b) and a == zlib.adler32(b), (off, m)
for _ in range(3): zt.dev_checksums(d.data_ptr(), n)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(20): zt.dev_checksums(d.data_ptr(), n)
torch.cuda.synchronize()
dt = (time.perf_counter() - t0) / 20
print(f"{os.environ.get('ZT_LIB', 'in-tree')}: ok; checksums 1 GiB {dt*1e3:.3f} ms per call ({n/dt/1e12:.2f} TB/s incl. call)", flush=True)
