"""Incompressible blocks skip the match search (deflate.hip classify_kernel):
a 32 KiB block whose sampled order-0 entropy is near 8 bits and that holds no
repeats inside its window is planned as a stored block (src/RawDeflate.ts:
122-153) without the chain walk.  The 16 ratio-gate windows: every random
(xorshift32) block is routed that way, no wordsalad / structured / source
block ever is; streams decode bit-exactly through the oracle's RawInflate and
Python's zlib.  Repeated random data and skewed (7-bit) random bytes must
still be searched / Huffman-coded."""
import random
import zlib

import pytest

from ratio_corpus import windows

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def zt():
    import ztamd

    assert ztamd.device_count() > 0, "no GPU visible"
    return ztamd


def _deflate_count(zt, data):
    zt.timing_enable(True)
    s = zt.deflate_raw(data)
    n = zt.timing_read()["blocks_unsearched"]
    zt.timing_enable(False)
    return s, n


@pytest.fixture(scope="module")
def wins(oracle):
    return windows(oracle)


@pytest.mark.parametrize("k", range(16))
def test_classify_ratio_windows(zt, oracle, wins, k):
    kind, label, w = wins[k]
    s, n = _deflate_count(zt, w)
    blocks = (len(w) + 32767) // 32768
    if kind == "xorshift32":
        assert n == blocks, (label, n)
        assert len(s) < len(w) * 1.0005
        out, ip = oracle.raw_inflate(s)
        assert out == w and ip == len(s)
    else:
        assert n == 0, (label, n)
        assert zlib.decompress(s, -15) == w


def test_classify_repeated_random(zt, oracle):
    r = oracle.gen("xorshift32", 77, 20 << 10)
    d = r * 6  # repeats 20 KiB back: inside the window
    s, n = _deflate_count(zt, d)
    assert n == 0  # every block holds a repeat of >= 12 KiB within the window
    assert zlib.decompress(s, -15) == d
    assert len(s) < len(d) * 0.3


def test_classify_skewed_bytes(zt):
    rng = random.Random(5)
    d = bytes(rng.getrandbits(7) for _ in range(256 << 10))  # ~7 bits per byte: Huffman saves ~1/8
    s, n = _deflate_count(zt, d)
    assert n == 0
    assert zlib.decompress(s, -15) == d
    assert len(s) < len(d) * 0.9


def test_classify_batch_and_fixed(zt, oracle):
    files = [oracle.gen("xorshift32", 300 + i, (i + 1) * 40000) for i in range(4)] + \
            [oracle.gen("wordsalad", 400 + i, (i + 1) * 40000) for i in range(4)]
    zt.timing_enable(True)
    members = zt.deflate_raw_batch(files)
    n = zt.timing_read()["blocks_unsearched"]
    zt.timing_enable(False)
    assert n == sum((len(f) + 32767) // 32768 for f in files[:4] if len(f) >= 4096)
    for f, m in zip(files, members):
        assert zlib.decompress(m, -15) == f
    # compressionType FIXED is never classified (fixed codes only, src/RawDeflate.ts:161-173)
    zt.timing_enable(True)
    s = zt.deflate_raw(files[0], compression_type=1)
    assert zt.timing_read()["blocks_unsearched"] == 0
    zt.timing_enable(False)
    assert zlib.decompress(s, -15) == files[0]


def test_classify_entropy_band(zt):
    # 240 equiprobable byte values: ~7.91 bits per byte, above the 4 KiB
    # sample's 7.85 cut but ~1 % below 8: the whole-block entropy (stage C)
    # must send every block to the search / Huffman coding, not store it
    rng = random.Random(11)
    d = bytes(rng.randrange(240) for _ in range(256 << 10))
    s, n = _deflate_count(zt, d)
    assert n == 0
    assert zlib.decompress(s, -15) == d
    assert len(s) < len(d) * 0.995


def test_classify_random_sample_over_filler(zt):
    # random bytes exactly where stage A samples (1 KiB at each quarter of a
    # block) over 4-bit filler without 8-byte repeats: the sample looks
    # incompressible, the block is not (stage C counts all of it)
    rng = random.Random(12)
    blocks = []
    for _ in range(4):
        blk = bytearray(rng.getrandbits(4) * 17 for _ in range(32768))
        for q in range(4):
            blk[q * 8192:q * 8192 + 1024] = bytes(rng.getrandbits(8) for _ in range(1024))
        blocks.append(bytes(blk))
    d = b"".join(blocks)
    s, n = _deflate_count(zt, d)
    assert n == 0
    assert zlib.decompress(s, -15) == d
    assert len(s) < len(d) * 0.75
