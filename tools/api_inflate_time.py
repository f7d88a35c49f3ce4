"""Host-API inflate of the bench corpus (1 GiB mixed, level 6): zt_inflate_raw
of the host stream into a library-allocated host output, PCIe included --
one warm call, then the best of 3 -- under the environment it runs in
(ZT_INF_NOPIPE, ZT_INF_PIECES are read once per process).
   usage: python tools/api_inflate_time.py [size_bytes]"""
import ctypes
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "zlib.ts_amd", "py"))
import torch  # noqa: E402
import ztamd as zt  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 30
d_in = torch.empty(n, dtype=torch.uint8, device="cuda")
zt.synth_dev("mixed", 7, d_in.data_ptr(), n)
d_c = torch.empty(zt.deflate_bound(n), dtype=torch.uint8, device="cuda")
dp = zt.DeflatePlan(n, level=6)
clen = dp.run(d_in.data_ptr(), n, d_c.data_ptr())
dp.close()
stream = d_c[:clen].cpu().numpy()
src = stream.ctypes.data_as(ctypes.c_void_p)
iopts = zt.InflateOpts(1, 0x8000, 0)
best = None
for rep in range(4):
    back = ctypes.POINTER(ctypes.c_uint8)()
    blen, ip = ctypes.c_size_t(), ctypes.c_size_t()
    t0 = time.perf_counter()
    zt._check(zt.lib.zt_inflate_raw(src, clen, 0, ctypes.byref(iopts), ctypes.byref(back), ctypes.byref(blen),
                                    ctypes.byref(ip)))
    dt = time.perf_counter() - t0
    assert blen.value == n and ip.value == clen
    zt.lib.zt_free(back)
    if rep:
        best = dt if best is None else min(best, dt)
env = {k: v for k, v in os.environ.items() if k.startswith("ZT_INF")}
print(f"api inflate {env}: {best * 1e3:.2f} ms = {n / best / 2**30:.2f} GiB/s (stream {clen} B)", flush=True)
