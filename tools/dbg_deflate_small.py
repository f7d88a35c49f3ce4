import sys, os
sys.path.insert(0, 'zlib.ts_amd/py'); sys.path.insert(0, 'tests')
import ztamd, zlib
n = int(sys.argv[1]); ct = int(sys.argv[2])
d = bytes((i * 7 + 3) & 0xFF for i in range(n)) if n < 100 else os.urandom(n)
out = ztamd.deflate_raw(d, compression_type=ct)
assert zlib.decompress(out, -15) == d
print('ok', n, ct, len(out), flush=True)
