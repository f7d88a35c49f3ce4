"""Stored runs next to Huffman blocks, built bit by bit.

The segment and batch inflate paths turn a stored payload of >= 1 KiB into
three run tokens (length << 16 with distance 0, then the payload's input
offset in two words; inflate_tok.hip) that expand_kernel writes straight from
the input.  These streams put the cases that token layout has to survive
into one unit:
  * a fixed-Huffman block right after the run whose short-distance matches
    copy from the run's last bytes (its last partial copy step);
  * a payload whose input offset has 16 low zero bits (the offset token then
    has the same bit pattern as a run token).
Expected output: Python's zlib on the same bytes (RFC 1951), and the bytes
the stream was built from.
"""
import random
import zlib

import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def zt():
    import ztamd

    assert ztamd.device_count() > 0, "no GPU visible"
    return ztamd


# RFC 1951 3.2.5: length / distance bases and extra bits
LEN_BASE = [3, 4, 5, 6, 7, 8, 9, 10, 11, 13, 15, 17, 19, 23, 27, 31, 35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195,
            227, 258]
LEN_EXTRA = [0] * 8 + [1] * 4 + [2] * 4 + [3] * 4 + [4] * 4 + [5] * 4 + [0]
DIST_BASE = [1, 2, 3, 4, 5, 7, 9, 13, 17, 25, 33, 49, 65, 97, 129, 193, 257, 385, 513, 769, 1025, 1537, 2049, 3073,
             4097, 6145, 8193, 12289, 16385, 24577]
DIST_EXTRA = [0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13]


class Bits:
    def __init__(self):
        self.out = bytearray()
        self.acc = 0
        self.n = 0

    def put(self, v, k):  # k bits of v, LSB first
        self.acc |= (v & ((1 << k) - 1)) << self.n
        self.n += k
        while self.n >= 8:
            self.out.append(self.acc & 0xFF)
            self.acc >>= 8
            self.n -= 8

    def code(self, c, k):  # Huffman code, MSB first
        r = 0
        for i in range(k):
            r |= ((c >> i) & 1) << (k - 1 - i)
        self.put(r, k)

    def align(self):
        if self.n:
            self.put(0, 8 - self.n)

    def pos(self):
        return len(self.out)


def fixed_sym(b, sym):
    if sym <= 143:
        b.code(0x30 + sym, 8)
    elif sym <= 255:
        b.code(0x190 + sym - 144, 9)
    elif sym <= 279:
        b.code(sym - 256, 7)
    else:
        b.code(0xC0 + sym - 280, 8)


def fixed_match(b, length, dist):
    i = max(k for k in range(29) if LEN_BASE[k] <= length)
    fixed_sym(b, 257 + i)
    b.put(length - LEN_BASE[i], LEN_EXTRA[i])
    j = max(k for k in range(30) if DIST_BASE[k] <= dist)
    b.code(j, 5)
    b.put(dist - DIST_BASE[j], DIST_EXTRA[j])


def stored(b, payload, final=False):
    b.put(1 if final else 0, 1)
    b.put(0, 2)
    b.align()
    n = len(payload)
    b.out += bytes([n & 0xFF, n >> 8, (~n) & 0xFF, ((~n) >> 8) & 0xFF])
    b.out += payload


def fixed_block(b, ops, out, final=False):
    """ops: ('lit', byte) or ('match', length, dist); appends the decoded bytes to out."""
    b.put(1 if final else 0, 1)
    b.put(1, 2)
    for op in ops:
        if op[0] == "lit":
            fixed_sym(b, op[1])
            out.append(op[1])
        else:
            _, length, dist = op
            fixed_match(b, length, dist)
            for _ in range(length):
                out.append(out[-dist])
    fixed_sym(b, 256)


def run_unit(b, out, rng, run_len):
    """A stored run of run_len bytes, then a fixed block whose matches copy from
    the run's tail (distances 1..run_len, overlapping copies), then a sync point."""
    payload = bytes(rng.getrandbits(8) for _ in range(run_len))
    stored(b, payload)
    out += payload
    ops = []
    for d in (1, 2, 3, 5, 7, 16, 31, 64, 100, 255, 511, 513):
        if d <= len(out):
            ops.append(("match", rng.choice([3, 4, 9, 17, 40, 258]), d))
        ops.append(("lit", rng.getrandbits(8)))
    fixed_block(b, ops, out)
    stored(b, b"")  # sync point (00 00 FF FF, byte-aligned)


def build(seed, aligned_at=65536, units=6):
    """A stream whose first unit's stored payload starts at input byte
    `aligned_at` (16 low zero bits), then further run units."""
    rng = random.Random(seed)
    b, out = Bits(), bytearray()
    # filler stored blocks so that the next stored block's header ends at aligned_at
    while True:
        left = aligned_at - 5 - b.pos() - 5  # this block's header + the next one's
        if left <= 65535:
            break
        pl = bytes(rng.getrandbits(8) for _ in range(60000))
        stored(b, pl)
        out += pl
    pl = bytes(rng.getrandbits(8) for _ in range(left))
    stored(b, pl)
    out += pl
    assert b.pos() + 5 == aligned_at
    run_unit(b, out, rng, 4096)  # payload at aligned_at
    for k in range(units):
        run_unit(b, out, rng, [1024, 1500, 3000, 8191, 1025, 2048][k % 6])
    fixed_block(b, [("match", 258, 1024), ("lit", 65)], out, final=True)
    b.align()
    return bytes(b.out), bytes(out)


@pytest.mark.parametrize("seed", [1, 2])
def test_stored_run_units_segment_path(zt, seed):
    s, d = build(seed)
    assert zlib.decompress(s, -15) == d
    out, ip = zt.inflate_raw(s)
    assert out == d and ip == len(s)
    # the same stream starting inside a larger buffer
    pre = b"\x55" * 77
    out2, ip2 = zt.inflate_raw(pre + s, index=len(pre))
    assert out2 == d and ip2 == len(pre) + len(s)


def test_stored_run_units_batch_path(zt):
    # stream 0 is packed at input offset 0, so its first run's payload sits at
    # input byte 65536 of the batch's device copy
    streams = []
    for seed in range(10):
        s, d = build(100 + seed, aligned_at=65536 if seed == 0 else 2048 + 64 * seed, units=3)
        assert zlib.decompress(s, -15) == d
        streams.append((s, d))
    res = zt.inflate_raw_batch([s for s, _ in streams])
    for (s, d), (st, out, ip) in zip(streams, res):
        assert st == 0 and out == d and ip == len(s)
