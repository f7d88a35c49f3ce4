"""CPU emulation of tok_huffman_simt (bitmap + merge-repair version) in
zlib.ts_amd/csrc/inflate_tok.hip, checked against a sequential decode.
Debug tool only."""
import random, sys, zlib
sys.path.insert(0, __import__('os').path.dirname(__file__))
from simt_emu import Bits, token, header, seq_body

L = 960
W = L // 32

def simt(b, b0, lt, dt, limit, stats):
    R = 0; out = []
    while True:
        stats['rounds'] += 1
        s = [R + l * L for l in range(64)]
        inr = [x < limit for x in s]
        bm = [[0] * W for _ in range(64)]
        end = list(s); ev = [0] * 64; flags = [0] * 64
        todo = list(inr); frm = list(s); repair = False
        for it in range(67):
            if it == 66: raise RuntimeError("no convergence")
            for l in range(64):
                if not todo[l]: continue
                pos = b0 + frm[l]
                cwi = (frm[l] - s[l]) >> 5; cw = 0
                if not repair: flags[l] = 0
                for x in range(cwi): bm[l][x] = 0
                while True:
                    p = pos - b0 - s[l]
                    wi = p >> 5
                    if wi != cwi:
                        bm[l][cwi] = cw
                        for x in range(cwi + 1, wi): bm[l][x] = 0
                        cwi = wi; cw = 0
                    if repair and (bm[l][wi] >> (p & 31)) & 1:
                        below = (1 << (p & 31)) - 1
                        bm[l][wi] = (cw & below) | (bm[l][wi] & ~below & 0xFFFFFFFF)
                        stats['merges'] += 1
                        break
                    cw |= 1 << (p & 31)
                    k, tk, nb, pos = token(b, pos, lt, dt)
                    stop = False
                    if k != 0 or pos - b0 > limit:
                        flags[l] = 1 if k > 0 else 2; ev[l] = s[l] + p; end[l] = pos - b0; stop = True
                    elif pos - b0 >= s[l] + L:
                        end[l] = pos - b0; flags[l] = 0; stop = True
                    if stop:
                        bm[l][cwi] = cw
                        for x in range(cwi + 1, W): bm[l][x] = 0
                        break
            t = [R] + end[:63]
            synced = []
            for l in range(64):
                tp = t[l] - s[l]
                synced.append(inr[l] and t[l] >= s[l] and tp < L and (bm[l][tp >> 5] >> (tp & 31)) & 1 == 1)
            U = [l for l in range(64) if not synced[l]]
            E = [l for l in range(64) if synced[l] and flags[l] != 0 and ev[l] >= t[l]]
            f = U[0] if U else 64; e = E[0] if E else 64
            if e < f:
                if flags[e] == 2: raise RuntimeError("invalid on true path")
                break
            if f == 64: break
            if not inr[f]: raise RuntimeError("past input")
            stats['repairs'] += sum(1 for l in range(64) if inr[l] and not synced[l])
            todo = [inr[l] and not synced[l] and s[l] <= t[l] < s[l] + L for l in range(64)]
            for l in range(64):
                if todo[l]: frm[l] = t[l]
            repair = True
        t = [R] + end[:63]
        E = [l for l in range(64) if flags[l] != 0 and ev[l] >= t[l] and inr[l]]
        e = E[0] if E else 64
        last = e if e < 64 else 63
        for l in range(last + 1):
            lo = t[l] - s[l]; hi = ev[l] - s[l] if l == e else L
            cnt = sum(1 for p in range(lo, hi) if (bm[l][p >> 5] >> (p & 31)) & 1)
            pos = b0 + t[l]
            for _ in range(cnt):
                k, tk, nb, pos = token(b, pos, lt, dt)
                assert k == 0
                out.append(tk)
            if l < last: assert pos - b0 == end[l], (l, pos - b0, end[l])
        if e < 64: return out, b0 + end[e]
        R = end[63]

def run(name, s):
    b = Bits(s + b"\0" * 16)
    pos = 0
    st = {'rounds': 0, 'repairs': 0, 'merges': 0}
    nblk = 0
    while True:
        bfinal, bt, lt, dt, pos = header(b, pos)
        ref, rpos = seq_body(b, pos, lt, dt)
        got, gpos = simt(b, pos, lt, dt, len(s) * 8 - pos, st)
        if got != ref or gpos != rpos:
            print(name, "block", nblk, "MISMATCH", len(got), len(ref), gpos, rpos); sys.exit(1)
        nblk += 1
        pos = rpos
        if bfinal: break
    print(name, nblk, "blocks OK", st)

rng = random.Random(5)
words = [b"the", b"of", b"deflate", b"huffman", b"window", b"gpu", b"lane", b"chunk"]
data = b" ".join(rng.choice(words) for _ in range(60000))
sdata = bytearray(); v = 0
for _ in range(40000):
    v = (v + rng.randrange(256) - 128) & 0xFFFFFFFF; sdata += v.to_bytes(4, 'little')
for name, d in [("words", data), ("structured", bytes(sdata)), ("tiny", b"hello hello hello")]:
    for lvl in (1, 6):
        c = zlib.compressobj(lvl, zlib.DEFLATED, -15)
        run(f"{name}-L{lvl}", c.compress(d) + c.flush())
