# Checksum kernel bound: CRC-32 + Adler-32 vs CRC-32 only vs Adler-32 only
# over 1 GiB device-resident bytes (zt_dev_checksums with a null output).
import ctypes, os, sys, time; sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', 'zlib.ts_amd', 'py'))
import torch, ztamd as zt
n = 1 << 30
d = torch.empty(n, dtype=torch.uint8, device="cuda")
zt.synth_dev("mixed", 3, d.data_ptr(), n)
c, a = ctypes.c_uint32(), ctypes.c_uint32()
for name, co, ao in [("both", ctypes.byref(c), ctypes.byref(a)), ("crc", ctypes.byref(c), None), ("adler", None, ctypes.byref(a))]:
    f = lambda: zt.lib.zt_dev_checksums(ctypes.c_void_p(d.data_ptr()), ctypes.c_size_t(n), 0, 1, co, ao, None)
    for _ in range(3): f()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(20): f()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / 20
    print(f"{os.environ.get('ZT_LIB', 'in-tree')} {name:6s} {dt*1e3:.3f} ms per call ({n/dt/1e12:.2f} TB/s)", flush=True)
