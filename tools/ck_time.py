# C1 checksum kernel timing: CRC-32 + Adler-32 over 1 GiB device-resident bytes
import os, sys, time; sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', 'zlib.ts_amd', 'py'))
import torch, ztamd as zt
n = 1 << 30
d = torch.empty(n, dtype=torch.uint8, device="cuda")
zt.synth_dev("mixed", 3, d.data_ptr(), n)
torch.cuda.synchronize()
for _ in range(3): zt.dev_checksums(d.data_ptr(), n)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(20): zt.dev_checksums(d.data_ptr(), n)
torch.cuda.synchronize()
dt = (time.perf_counter() - t0) / 20
print(f"checksums 1 GiB: {dt*1e3:.3f} ms per call ({n/dt/1e12:.2f} TB/s incl. call)", flush=True)
