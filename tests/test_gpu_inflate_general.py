"""General parallel inflate (csrc/inflate_gen.hip): streams WITHOUT sync
points -- the reference's own RawDeflate output (the whole input as ONE
dynamic block, src/RawDeflate.ts:105-107) and zlib raw streams (many blocks,
none byte-aligned) -- decoded by many waves from speculative bit offsets.
Every output is checked bit-exact against the pinned oracle's RawInflate
(the reference's algorithm restated, tests/golden pins it) or zlib, and the
`inflate_paths` counters show the general path (not the one-wave fallback)
produced it."""
import random
import zlib

import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def zt():
    import ztamd

    assert ztamd.device_count() > 0, "no GPU visible"
    return ztamd


def _mixed(oracle, n, seed):
    kinds = ["wordsalad", "xorshift32", "structured"]
    out, i = [], 0
    while sum(len(x) for x in out) < n:
        out.append(oracle.gen(kinds[(seed + i) % 3], seed * 101 + i, 1 << 20))
        i += 1
    return b"".join(out)[:n]


def _general(zt, stream, index=0):
    before = zt.timing_read()["inflate_paths"]
    out, ip = zt.inflate_raw(stream, index=index)
    after = zt.timing_read()["inflate_paths"]
    return out, ip, after[1] - before[1], after[2] - before[2]


def _zraw(data, level=6, strategy=zlib.Z_DEFAULT_STRATEGY, mem=8):
    c = zlib.compressobj(level, zlib.DEFLATED, -15, mem, strategy)
    return c.compress(data) + c.flush()


@pytest.mark.parametrize("size", [1 << 20, 8 << 20])
def test_reference_single_block(zt, oracle, size):
    """The reference's RawDeflate writes one dynamic block; the engine decodes
    it with many waves, bit-exact, with the reference's end ip."""
    data = _mixed(oracle, size, 3)
    s, _ = oracle.raw_deflate(data)
    out, ip, gen, one = _general(zt, s)
    assert out == data and ip == len(s)
    assert gen == 1 and one == 0


def test_reference_single_block_64mib(zt, oracle):
    """SURVEY 8(d) C2 / VERDICT r1 item 5: a 64 MiB reference-style stream."""
    data = _mixed(oracle, 64 << 20, 5)
    s, _ = oracle.raw_deflate(data)
    ref, rip = oracle.raw_inflate(s)
    assert ref == data and rip == len(s)
    out, ip, gen, one = _general(zt, s)
    assert out == data and ip == len(s)
    assert gen == 1 and one == 0


@pytest.mark.parametrize("level", [1, 6, 9])
def test_zlib_levels(zt, oracle, level):
    data = _mixed(oracle, 16 << 20, level)
    s = _zraw(data, level)
    out, ip, gen, one = _general(zt, s)
    assert out == data and ip == len(s)
    assert gen == 1 and one == 0


@pytest.mark.parametrize("strategy", ["fixed", "huffman", "rle", "filtered"])
def test_zlib_strategies(zt, oracle, strategy):
    st = {"fixed": zlib.Z_FIXED, "huffman": zlib.Z_HUFFMAN_ONLY, "rle": zlib.Z_RLE,
          "filtered": zlib.Z_FILTERED}[strategy]
    data = _mixed(oracle, 4 << 20, 7)
    s = _zraw(data, 6, st)
    out, ip, gen, one = _general(zt, s)
    assert out == data and ip == len(s)
    assert gen == 1


def test_zlib_incompressible(zt):
    """zlib writes stored blocks for random data: LEN / NLEN candidates."""
    data = random.Random(11).randbytes(6 << 20)
    s = _zraw(data, 6)
    out, ip, gen, one = _general(zt, s)
    assert out == data and ip == len(s)


def test_reference_random_single_block(zt):
    """Random bytes in ONE dynamic block (literal codes of 8-9 bits, slow to
    resynchronise): the links that fail are redone exactly."""
    import zt_oracle

    o = zt_oracle.Oracle()
    data = random.Random(12).randbytes(2 << 20)
    s, _ = o.raw_deflate(data)
    out, ip, gen, one = _general(zt, s)
    assert out == data and ip == len(s)


def test_index_and_trailing_bytes(zt, oracle):
    """RawInflate `index` and bytes after the stream (a gzip trailer): the
    output and the end ip are exact."""
    data = _mixed(oracle, 3 << 20, 9)
    pre = b"\x1f\x8b\x08\x00junkheader"
    s = pre + _zraw(data, 6) + b"TRAILER!" * 4
    out, ip, gen, one = _general(zt, s, index=len(pre))
    assert out == data and ip == len(s) - 32


def test_concatenated_long_matches(zt):
    """Highly repetitive input: long match chains across every segment
    boundary resolve through the window markers."""
    unit = b"".join(bytes([i % 251, (i * 7) % 256]) * 3 for i in range(4000))
    data = unit * 300  # 7.2 MB, period 24000 bytes
    s = _zraw(data, 9)
    out, ip, gen, one = _general(zt, s)
    assert out == data and ip == len(s)
    s2 = _zraw(b"\x00" * (12 << 20) + data[:1 << 20], 6)
    out, ip, gen, one = _general(zt, s2)
    assert out == b"\x00" * (12 << 20) + data[:1 << 20]


@pytest.mark.parametrize("seed", range(6))
def test_corrupt_streams_match_one_wave(zt, oracle, seed):
    """Corrupted streams: the general path either decodes exactly what the
    sequential one-wave decoder decodes, or raises the same error."""
    import ztamd

    rng = random.Random(seed)
    data = _mixed(oracle, 2 << 20, seed)
    s = bytearray(_zraw(data, 6) if seed % 2 else oracle.raw_deflate(data)[0])
    for _ in range(1 + seed):
        i = rng.randrange(len(s) // 4, len(s))
        s[i] ^= 1 << rng.randrange(8)
    s = bytes(s)
    st, want, wip = zt.inflate_raw_batch([s])[0]
    try:
        out, ip = zt.inflate_raw(s)
    except ztamd.ZtError as e:
        assert st != 0 and e.code == st
        return
    assert st == 0 and out == want and ip == wip
