# Which deflate configurations produce a stream that does not round-trip?
import os, sys, zlib; sys.path.insert(0, 'tests'); sys.path.insert(0, 'zlib.ts_amd/py')
import zt_oracle, ztamd as zt
o = zt_oracle.Oracle()
for kind, n in [("xorshift32", 65539), ("xorshift32", 4096), ("wordsalad", 65539), ("structured", 100000)]:
    d = o.gen(kind, 1, n)
    s = zt.deflate_raw(d)
    try:
        ok = zlib.decompress(s, -15) == d
    except Exception as e:
        ok = str(e)
    print(kind, n, len(s), ok, s[:16].hex(), s[-16:].hex(), flush=True)
