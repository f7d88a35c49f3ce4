"""Debug: tokens of a raw DEFLATE stream's first (dynamic) block decoded from a
given bit position with the block's tables (pure Python, small ranges only).
   usage: from pyinflate_tokens import tokens_from"""
ORD = [16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15]
LB = [3, 4, 5, 6, 7, 8, 9, 10, 11, 13, 15, 17, 19, 23, 27, 31, 35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 258]
LE = [0] * 8 + [1] * 4 + [2] * 4 + [3] * 4 + [4] * 4 + [5] * 4 + [0]
DB = [1, 2, 3, 4, 5, 7, 9, 13, 17, 25, 33, 49, 65, 97, 129, 193, 257, 385, 513, 769, 1025, 1537, 2049, 3073, 4097,
      6145, 8193, 12289, 16385, 24577]
DE = [0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13]


class Bits:
    def __init__(self, s):
        self.s = s

    def get(self, pos, n):
        v = 0
        for k in range(n):
            v |= ((self.s[(pos + k) >> 3] >> ((pos + k) & 7)) & 1) << k
        return v


def build(lens):
    d = {}
    code = 0
    bl = [0] * 16
    for l in lens:
        if l:
            bl[l] += 1
    nxt = [0] * 16
    for b in range(1, 16):
        code = (code + bl[b - 1]) << 1
        nxt[b] = code
    for sym, l in enumerate(lens):
        if l:
            d[(l, nxt[l])] = sym
            nxt[l] += 1
    return d


def dec(bits, pos, d):
    code = 0
    for l in range(1, 16):
        code = (code << 1) | bits.get(pos + l - 1, 1)
        if (l, code) in d:
            return d[(l, code)], l
    raise ValueError("bad code")


def tables(s, hdr=0):
    b = Bits(s)
    pos = hdr + 3
    hlit = b.get(pos, 5) + 257
    hd = b.get(pos + 5, 5) + 1
    hc = b.get(pos + 10, 4) + 4
    pos += 14
    cl = [0] * 19
    for i in range(hc):
        cl[ORD[i]] = b.get(pos, 3)
        pos += 3
    cd = build(cl)
    L = []
    while len(L) < hlit + hd:
        sy, ln = dec(b, pos, cd)
        pos += ln
        if sy < 16:
            L.append(sy)
        elif sy == 16:
            L += [L[-1]] * (3 + b.get(pos, 2))
            pos += 2
        elif sy == 17:
            L += [0] * (3 + b.get(pos, 3))
            pos += 3
        else:
            L += [0] * (11 + b.get(pos, 7))
            pos += 7
    return build(L[:hlit]), build(L[hlit:]), pos


def tokens_from(s, pos, count, hdr=0):
    """[(bit position, token as the engine encodes it: byte or len << 16 | dist)]"""
    lt, dt, _ = tables(s, hdr)
    b = Bits(s)
    out = []
    for _ in range(count):
        p0 = pos
        sy, ln = dec(b, pos, lt)
        pos += ln
        if sy < 256:
            out.append((p0, sy))
        elif sy == 256:
            out.append((p0, -1))
            break
        else:
            i = sy - 257
            L = LB[i] + b.get(pos, LE[i])
            pos += LE[i]
            ds, ln = dec(b, pos, dt)
            pos += ln
            D = DB[ds] + b.get(pos, DE[ds])
            pos += DE[ds]
            out.append((p0, (L << 16) | D))
    return out
