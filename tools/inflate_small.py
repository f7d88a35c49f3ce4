import sys, zlib; sys.path.insert(0,'tests'); sys.path.insert(0,'zlib.ts_amd/py')
import zt_oracle, ztamd
o = zt_oracle.Oracle()
d = o.gen("wordsalad", 7, 1 << 20)
s = zlib.compress(d, 6)[2:-4]
out, ip = ztamd.inflate_raw(s)
assert out == d
import struct
toks = 0
print('stream', len(s), 'out', len(d))
