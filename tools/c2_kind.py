# C2 per-corpus latency: batch of 64 copies of one reference-deflated 64 KiB stream
import os, sys, time
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, '..', 'zlib.ts_amd', 'py')); sys.path.insert(0, os.path.join(HERE, '..', 'tests'))
import ztamd as zt, zt_oracle, zlib
o = zt_oracle.Oracle()
for kind in ("wordsalad", "structured", "xorshift32"):
    raw = o.gen(kind, 500, 65536)
    for src, s in (("ref", o.raw_deflate(raw)[0]), ("zlib6", zlib.compress(raw, 6)[2:-4])):
        streams = [s] * 64
        zt.inflate_raw_batch(streams)
        t0 = time.perf_counter(); r = zt.inflate_raw_batch(streams); t1 = time.perf_counter()
        assert r[0][1] == raw
        print(f"{kind:10s} {src:5s} in {len(s):6d} B: {1e3*(t1-t0):.2f} ms", flush=True)
