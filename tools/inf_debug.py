# Which inputs leave the two-phase inflate (run with ZT_INF_DEBUG=1)?
import sys; sys.path.insert(0, 'tests'); sys.path.insert(0, 'zlib.ts_amd/py')
import zt_oracle, ztamd as zt
o = zt_oracle.Oracle()
cases = {"wordsalad": o.gen("wordsalad", 21, (1 << 20) + 777), "zeros": b"\0" * (1 << 20) + b"x",
         "abc": b"abc" * 400000, "random": o.gen("xorshift32", 22, 300001) * 2, "structured": o.gen("structured", 23, 1 << 20),
         "ramp": bytes(range(256)) * 3000}
for k, d in cases.items():
    s = zt.deflate_raw(d)
    zt.timing_enable(True)
    out, ip = zt.inflate_raw(s)
    t = zt.timing_read(); zt.timing_enable(False)
    print(k, len(d), len(s), "ok" if out == d and ip == len(s) else "MISMATCH", "two-phase" if t["inflate_toks"] else "fallback", flush=True)
