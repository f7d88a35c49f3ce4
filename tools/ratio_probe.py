import sys, time; sys.path.insert(0,'tests'); sys.path.insert(0,'zlib.ts_amd/py')
import zt_oracle, ztamd, zlib
o = zt_oracle.Oracle()
for kind in ["wordsalad", "xorshift32", "structured"]:
    d = o.gen(kind, 4, 1 << 20)
    ref = len(o.raw_deflate(d)[0])
    row = [kind, ref, 'zlib6 %.4f' % (len(zlib.compress(d, 6)) / ref), 'zlib9 %.4f' % (len(zlib.compress(d, 9)) / ref)]
    for lv in (1, 4, 6, 8, 9):
        ztamd.deflate_raw(d, level=lv)
        t = time.time(); s = ztamd.deflate_raw(d, level=lv); dt = time.time() - t
        row.append('L%d %.4f' % (lv, len(s) / ref))
    print(*row, flush=True)
