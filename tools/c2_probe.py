# C2 breakdown: batch RawInflate of 4096 x 64 KiB streams, C call vs Python wrapping
import os, sys, time, ctypes
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, '..', 'zlib.ts_amd', 'py')); sys.path.insert(0, os.path.join(HERE, '..', 'tests'))
import ztamd as zt, zt_oracle
o = zt_oracle.Oracle()
pieces = []
for i in range(64):
    kind = ["wordsalad", "structured", "xorshift32"][i % 3]
    raw = o.gen(kind, 500 + i, 65536)
    pieces.append(o.raw_deflate(raw)[0])
for count in (64, 512, 4096):
    streams = [pieces[i % 64] for i in range(count)]
    k = count
    bufs = [zt._cbuf(s) for s in streams]
    ptrs = (ctypes.c_void_p * k)(*[ctypes.addressof(b) for b, _ in bufs])
    lens = (ctypes.c_size_t * k)(*[n for _, n in bufs])
    outs = (ctypes.POINTER(ctypes.c_uint8) * k)()
    olens = (ctypes.c_size_t * k)(); ips = (ctypes.c_size_t * k)(); st = (ctypes.c_int * k)()
    opts = zt.InflateOpts(1, 0x8000, 0)
    for rep in range(3):
        t0 = time.perf_counter()
        rc = zt.lib.zt_inflate_raw_batch(ptrs, lens, k, ctypes.byref(opts), outs, olens, ips, st)
        t1 = time.perf_counter()
        for i in range(k): zt.lib.zt_free(outs[i])
    print(f"count {count}: C call {1e3*(t1-t0):.2f} ms -> {count*65536/(t1-t0)/2**30:.3f} GiB/s", flush=True)
t0 = time.perf_counter(); zt.inflate_raw_batch(streams); t1 = time.perf_counter()
print(f"python wrapper 4096: {1e3*(t1-t0):.2f} ms", flush=True)
