"""Host-API deflate of the bench corpus (1 GiB mixed, level 6): zt_deflate_raw
of a pageable host copy into a library-allocated host stream, PCIe included --
one warm call, then the best of 3 -- under the environment it runs in
(ZT_DF_PIECES is read once per process).  The stream is checked against the
device plan's.
   usage: python tools/api_deflate_time.py [size_bytes]"""
import ctypes
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "zlib.ts_amd", "py"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import ztamd as zt  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 30
d_in = torch.empty(n, dtype=torch.uint8, device="cuda")
zt.synth_dev("mixed", 7, d_in.data_ptr(), n)
d_c = torch.empty(zt.deflate_bound(n), dtype=torch.uint8, device="cuda")
dp = zt.DeflatePlan(n, level=6)
clen = dp.run(d_in.data_ptr(), n, d_c.data_ptr())
dp.close()
ref = d_c[:clen].cpu().numpy()
host = d_in.cpu().numpy()
src = host.ctypes.data_as(ctypes.c_void_p)
opts = zt.DeflateOpts(2, 0, 6)
best = None
for rep in range(4):
    out = ctypes.POINTER(ctypes.c_uint8)()
    olen = ctypes.c_size_t()
    t0 = time.perf_counter()
    zt._check(zt.lib.zt_deflate_raw(src, n, ctypes.byref(opts), ctypes.byref(out), ctypes.byref(olen)))
    dt = time.perf_counter() - t0
    got = np.ctypeslib.as_array(out, shape=(olen.value,))
    assert olen.value == clen and np.array_equal(got, ref), "API stream differs from the device plan's"
    zt.lib.zt_free(out)
    if rep:
        best = dt if best is None else min(best, dt)
env = {k: v for k, v in os.environ.items() if k.startswith("ZT_DF")}
print(f"api deflate {env}: {best * 1e3:.2f} ms = {n / best / 2**30:.2f} GiB/s (stream {clen} B)", flush=True)
