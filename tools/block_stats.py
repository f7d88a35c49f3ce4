# Per-block accounting of this engine's deflate output: header bits (BTYPE..code
# lengths), body bits, sync-marker bits, per corpus (4 MiB windows, level 6).
import os, sys
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, '..', 'zlib.ts_amd', 'py')); sys.path.insert(0, os.path.join(HERE, '..', 'tests'))
import ztamd as zt, zt_oracle

class Bits:
    def __init__(s, b): s.b, s.p = b, 0
    def get(s, n):
        v = 0
        for i in range(n):
            v |= ((s.b[(s.p + i) >> 3] >> ((s.p + i) & 7)) & 1) << i
        s.p += n
        return v

def codes(lengths):
    # canonical decode map: (len, code) -> symbol
    bl = [0] * 16
    for l in lengths:
        if l: bl[l] += 1
    nxt, c = [0] * 16, 0
    for l in range(1, 16):
        c = (c + bl[l - 1]) << 1
        nxt[l] = c
    m = {}
    for sym, l in enumerate(lengths):
        if l:
            m[(l, nxt[l])] = sym
            nxt[l] += 1
    return m

def sym(bits, m):
    c, l = 0, 0
    while True:
        c = (c << 1) | bits.get(1); l += 1
        if (l, c) in m: return m[(l, c)]
        if l > 15: raise ValueError("bad code")

LB = [3,4,5,6,7,8,9,10,11,13,15,17,19,23,27,31,35,43,51,59,67,83,99,115,131,163,195,227,258]
LE = [0,0,0,0,0,0,0,0,1,1,1,1,2,2,2,2,3,3,3,3,4,4,4,4,5,5,5,5,0]
DE = [0,0,0,0,1,1,2,2,3,3,4,4,5,5,6,6,7,7,8,8,9,9,10,10,11,11,12,12,13,13]

def analyse(s):
    b = Bits(s); hdr = body = stored = 0; nblk = 0
    while True:
        p0 = b.p
        final = b.get(1); bt = b.get(2)
        if bt == 0:
            b.p = (b.p + 7) & ~7
            ln = b.get(16); b.get(16); b.p += 8 * ln
            stored += b.p - p0
        elif bt == 2:
            nblk += 1
            hlit = b.get(5) + 257; hdist = b.get(5) + 1; hclen = b.get(4) + 4
            order = [16,17,18,0,8,7,9,6,10,5,11,4,12,3,13,2,14,1,15]
            cl = [0] * 19
            for i in range(hclen): cl[order[i]] = b.get(3)
            cm = codes(cl); lens = []
            while len(lens) < hlit + hdist:
                x = sym(b, cm)
                if x < 16: lens.append(x)
                elif x == 16: lens += [lens[-1]] * (3 + b.get(2))
                elif x == 17: lens += [0] * (3 + b.get(3))
                else: lens += [0] * (11 + b.get(7))
            hdr += b.p - p0; q = b.p
            lm, dm = codes(lens[:hlit]), codes(lens[hlit:])
            while True:
                x = sym(b, lm)
                if x == 256: break
                if x > 256:
                    b.get(LE[x - 257]); d = sym(b, dm); b.get(DE[d])
            body += b.p - q
        else:
            raise ValueError("unexpected block type %d" % bt)
        if final: break
    return nblk, hdr // 8, body // 8, stored // 8

o = zt_oracle.Oracle()
n = 4 << 20
for kind in ("wordsalad", "structured"):
    raw = o.gen(kind, 3, n)
    s = zt.deflate_raw(raw, level=6)
    nb, h, bd, st = analyse(s)
    print(f"{kind}: stream {len(s)} B, {nb} blocks, headers {h} B ({100*h/len(s):.2f} %), bodies {bd} B, "
          f"stored/markers {st} B ({100*st/len(s):.2f} %); header per block {h/nb:.0f} B", flush=True)
