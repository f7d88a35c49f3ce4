"""Debug helper: decode a raw DEFLATE stream into (kind, ...) tokens.

Pure Python, small inputs only.  Used to inspect what the GPU encoder emitted.
"""
import sys

LBASE = [3, 4, 5, 6, 7, 8, 9, 10, 11, 13, 15, 17, 19, 23, 27, 31, 35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227,
         258]
LEXT = [0] * 8 + [1] * 4 + [2] * 4 + [3] * 4 + [4] * 4 + [5] * 4 + [0]
DBASE = [1, 2, 3, 4, 5, 7, 9, 13, 17, 25, 33, 49, 65, 97, 129, 193, 257, 385, 513, 769, 1025, 1537, 2049, 3073, 4097,
         6145, 8193, 12289, 16385, 24577]
DEXT = [0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13]
ORDER = [16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15]


class Bits:
    def __init__(self, b):
        self.b, self.pos = b, 0

    def get(self, n):
        v = 0
        for i in range(n):
            v |= ((self.b[self.pos >> 3] >> (self.pos & 7)) & 1) << i
            self.pos += 1
        return v


def table(lens):
    codes = {}
    code = 0
    for l in range(1, 16):
        for s, ln in enumerate(lens):
            if ln == l:
                codes[(l, code)] = s
                code += 1
        code <<= 1
    return codes


def sym(bits, t):
    code = 0
    for l in range(1, 16):
        code = (code << 1) | bits.get(1)
        if (l, code) in t:
            return t[(l, code)]
    raise ValueError("bad code at bit %d" % bits.pos)


def tokens(stream):
    bits = Bits(stream)
    out = []
    data = bytearray()
    final = 0
    while not final:
        final = bits.get(1)
        bt = bits.get(2)
        out.append(("block", bt, final, bits.pos))
        if bt == 0:
            bits.pos = (bits.pos + 7) & ~7
            ln = bits.get(16)
            bits.get(16)
            for _ in range(ln):
                data.append(bits.get(8))
            out.append(("stored", ln))
            continue
        if bt == 1:
            lt = table([8] * 144 + [9] * 112 + [7] * 24 + [8] * 8)
            dt = table([5] * 30)
        else:
            hlit, hdist, hclen = bits.get(5) + 257, bits.get(5) + 1, bits.get(4) + 4
            cl = [0] * 19
            for i in range(hclen):
                cl[ORDER[i]] = bits.get(3)
            ct = table(cl)
            lens = []
            while len(lens) < hlit + hdist:
                s = sym(bits, ct)
                if s < 16:
                    lens.append(s)
                elif s == 16:
                    lens += [lens[-1]] * (3 + bits.get(2))
                elif s == 17:
                    lens += [0] * (3 + bits.get(3))
                else:
                    lens += [0] * (11 + bits.get(7))
            lt, dt = table(lens[:hlit]), table(lens[hlit:])
        while True:
            s = sym(bits, lt)
            if s < 256:
                out.append(("lit", len(data), s))
                data.append(s)
            elif s == 256:
                break
            else:
                L = LBASE[s - 257] + bits.get(LEXT[s - 257])
                ds = sym(bits, dt)
                D = DBASE[ds] + bits.get(DEXT[ds])
                out.append(("match", len(data), L, D))
                for _ in range(L):
                    data.append(data[-D])
    return out, bytes(data)


if __name__ == "__main__":
    s = open(sys.argv[1], "rb").read()
    toks, data = tokens(s)
    for t in toks:
        print(t)
