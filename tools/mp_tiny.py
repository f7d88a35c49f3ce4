import sys, os
sys.path.insert(0, 'zlib.ts_amd/py')
import ztamd as zt
for n in [1, 3, 100, 5000]:
    d = bytes((i * 7) & 255 for i in range(n))
    s = zt.deflate_raw(d)
    print("n", n, "->", len(s), flush=True)
