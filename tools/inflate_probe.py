import sys, time, zlib; sys.path.insert(0,'tests'); sys.path.insert(0,'zlib.ts_amd/py')
import zt_oracle, ztamd, torch
o = zt_oracle.Oracle()
for kind in ["wordsalad", "xorshift32", "structured"]:
    d = o.gen(kind, 7, 16 << 20)
    s = zlib.compress(d, 6)[2:-4]
    ztamd.inflate_raw(s)
    t0 = time.time(); out, ip = ztamd.inflate_raw(s); dt = time.time() - t0
    assert out == d
    print(kind, 'single wave: %.1f MB/s (incl. PCIe)' % (len(d) / dt / 1e6), flush=True)
# C2: 4096 x 64 KiB
items = []
for i in range(4096):
    d = o.gen("xorshift32" if i % 2 == 0 else "wordsalad", 100 + i, 65536)
    items.append(zlib.compress(d, 6)[2:-4])
ztamd.inflate_raw_batch(items[:64])
t0 = time.time(); res = ztamd.inflate_raw_batch(items); dt = time.time() - t0
print('C2 batch 4096x64KiB: %.2f GiB/s (host API incl. PCIe)' % (4096 * 65536 / dt / 2**30))
