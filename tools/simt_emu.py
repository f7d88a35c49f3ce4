"""CPU emulation of tokenize_kernel's SIMT block-body decode (inflate_tok.hip):
speculative per-lane decoding in rounds of 64 x SP_LANE_BITS, boundary
matching, repair, exact counts.  Checks it against a plain sequential decode
of the same blocks (zlib streams).  Debug tool, not part of the product."""
import random, sys, zlib

SP_K, LB = 8, 448
LBASE = [3,4,5,6,7,8,9,10,11,13,15,17,19,23,27,31,35,43,51,59,67,83,99,115,131,163,195,227,258]
LEXT = [0]*8+[1]*4+[2]*4+[3]*4+[4]*4+[5]*4+[0]
DBASE = [1,2,3,4,5,7,9,13,17,25,33,49,65,97,129,193,257,385,513,769,1025,1537,2049,3073,4097,6145,8193,12289,16385,24577]
DEXT = [0,0,0,0,1,1,2,2,3,3,4,4,5,5,6,6,7,7,8,8,9,9,10,10,11,11,12,12,13,13]

class Bits:
    def __init__(s, data): s.v = int.from_bytes(data, 'little'); s.n = len(data) * 8
    def get(s, pos, k): return (s.v >> pos) & ((1 << k) - 1)

def build(lens):
    # map (len, reversed code) -> sym
    cnt = [0]*16
    for l in lens:
        if l: cnt[l] += 1
    code, nxt = 0, [0]*16
    for l in range(1, 16):
        code = (code + cnt[l-1]) << 1 if l > 1 else 0
        nxt[l] = code
    t = {}
    for s_, l in enumerate(lens):
        if l:
            c = nxt[l]; nxt[l] += 1
            r = int(bin(c)[2:].zfill(l)[::-1], 2)
            t[(l, r)] = s_
    return t

def dec_sym(b, pos, t):
    for l in range(1, 16):
        if (l, b.get(pos, l)) in t: return t[(l, b.get(pos, l))], l
    return None, 0

def token(b, pos, lt, dt):
    """-> (kind, tok, nbytes, newpos): kind 0 token, 1 eob, -1 invalid"""
    s_, l = dec_sym(b, pos, lt)
    if s_ is None: return -1, 0, 0, pos
    pos += l
    if s_ < 256: return 0, s_, 1, pos
    if s_ == 256: return 1, 0, 0, pos
    ls = s_ - 257
    if ls >= 29: ls = 28
    ln = LBASE[ls] + b.get(pos, LEXT[ls]); pos += LEXT[ls]
    d, l2 = dec_sym(b, pos, dt)
    if d is None or d >= 30: return -1, 0, 0, pos
    pos += l2
    dist = DBASE[d] + b.get(pos, DEXT[d]); pos += DEXT[d]
    return 0, (ln << 16) | dist, ln, pos

CLO = [16,17,18,0,8,7,9,6,10,5,11,4,12,3,13,2,14,1,15]
def header(b, pos):
    bfinal = b.get(pos, 1); bt = b.get(pos+1, 2); pos += 3
    if bt == 1:
        ll = [8]*144+[9]*112+[7]*24+[8]*8
        return bfinal, bt, build(ll), build([5]*30), pos
    assert bt == 2, bt
    hlit = b.get(pos,5)+257; hdist = b.get(pos+5,5)+1; hclen = b.get(pos+10,4)+4; pos += 14
    cl = [0]*19
    for i in range(hclen): cl[CLO[i]] = b.get(pos,3); pos += 3
    ct = build(cl); L = []
    while len(L) < hlit+hdist:
        s_, l = dec_sym(b, pos, ct); pos += l
        if s_ < 16: L.append(s_)
        elif s_ == 16: L += [L[-1]]*(3+b.get(pos,2)); pos += 2
        elif s_ == 17: L += [0]*(3+b.get(pos,3)); pos += 3
        else: L += [0]*(11+b.get(pos,7)); pos += 7
    return bfinal, bt, build(L[:hlit]), build(L[hlit:hlit+hdist]), pos

def seq_body(b, pos, lt, dt):
    toks = []
    while True:
        k, tk, nb, pos = token(b, pos, lt, dt)
        assert k >= 0
        if k == 1: return toks, pos
        toks.append(tk)

def simt_body(b, b0, lt, dt, limit):
    R, out = 0, []
    stats = {"rounds": 0, "repairs": 0}
    while True:
        stats["rounds"] += 1
        st = [R + l*LB for l in range(64)]; s_next = [x + LB for x in st]
        inr = [x < limit for x in st]
        st_ = list(st)
        end = [0]*64; ntok=[0]*64; nby=[0]*64; flags=[0]*64; bpos=[[None]*SP_K for _ in range(64)]; bby=[[0]*SP_K for _ in range(64)]; nrec=[0]*64
        todo = list(inr); lanetoks = [[] for _ in range(64)]
        for rnd in range(70):
            for l in range(64):
                if not todo[l]: continue
                pos = b0 + st_[l]; ntok[l]=nby[l]=nrec[l]=flags[l]=0; lanetoks[l]=[]
                while True:
                    if nrec[l] < SP_K: bpos[l][nrec[l]] = pos - b0; bby[l][nrec[l]] = nby[l]; nrec[l] += 1
                    k, tk, nb, pos = token(b, pos, lt, dt)
                    if k < 0 or pos - b0 > limit: flags[l]=2; end[l]=pos-b0; break
                    if k == 1: flags[l]=1; end[l]=pos-b0; break
                    ntok[l]+=1; nby[l]+=nb; lanetoks[l].append(tk)
                    if pos - b0 >= s_next[l]: end[l]=pos-b0; break
            prev = [R] + end[:63]
            kk = [-1]*64
            for l in range(64):
                if inr[l]:
                    for k in range(nrec[l]):
                        if bpos[l][k] == prev[l]: kk[l]=k; break
            fail=-1; last=-1
            for l in range(64):
                if kk[l] < 0: fail=l; break
                if flags[l]==2: raise RuntimeError("invalid on true path")
                last=l
                if flags[l]==1: break
            if fail < 0: break
            stats["repairs"] += 1
            todo=[False]*64; todo[fail]=True; st_[fail]=prev[fail]
        eob = flags[last]==1
        for l in range(last+1):
            out += lanetoks[l][kk[l]:]
        if eob: return out, b0 + end[last], stats
        R = end[last]

def main():
    rng = random.Random(5)
    words = [b"the", b"of", b"deflate", b"huffman", b"window", b"gpu", b"lane", b"chunk"]
    data = b" ".join(rng.choice(words) for _ in range(60000))
    sdata = bytearray()
    v = 0
    for _ in range(40000):
        v = (v + rng.randrange(256) - 128) & 0xFFFFFFFF; sdata += v.to_bytes(4, 'little')
    for name, d in [("words", data), ("structured", bytes(sdata))]:
        c = zlib.compressobj(6, zlib.DEFLATED, -15)
        s = c.compress(d) + c.flush()
        b = Bits(s + b"\0"*16)
        pos = 0
        while True:
            bfinal, bt, lt, dt, pos = header(b, pos)
            ref, rpos = seq_body(b, pos, lt, dt)
            got, gpos, st = simt_body(b, pos, lt, dt, len(s)*8 - pos)
            ok = got == ref and gpos == rpos
            print(name, "block", len(ref), "tokens", "OK" if ok else "MISMATCH", st, gpos, rpos)
            if not ok:
                for i,(x,y) in enumerate(zip(got, ref)):
                    if x != y: print(" first diff at", i); break
                sys.exit(1)
            pos = rpos
            if bfinal: break

main()
