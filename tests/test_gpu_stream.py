"""Streaming inflate (src/RawInflateStream.ts:67-120):
zt_inflate_raw_resume through ztamd.RawInflateStream.  A stream fed in
pieces -- every call given the whole input received so far, as the
reference's callers do -- yields, concatenated, exactly the oracle's decode
of the whole stream; running out of input is never an error; a corrupt
stream fails with the reference's message."""
import random
import zlib

import pytest

pytestmark = pytest.mark.gpu


def stream_in_pieces(stream, cuts):
    import ztamd

    st = ztamd.RawInflateStream()
    parts = [st.decompress(stream[:end]) for end in cuts]
    return parts, st


def raw(data, level=6, strategy=zlib.Z_DEFAULT_STRATEGY, mem=8):
    c = zlib.compressobj(level, zlib.DEFLATED, -15, mem, strategy)
    return c.compress(data) + c.flush()


def corpora(oracle):
    text = oracle.gen("wordsalad", 11, 400_000)
    mixed = text[:150_000] + oracle.gen("xorshift32", 11, 70_000) + oracle.gen("structured", 11, 120_000)
    return text, mixed


@pytest.mark.parametrize("kind", ["zlib6", "zlib1", "zlib9", "stored", "fixed", "huffman_only", "reference", "engine"])
def test_stream_pieces_equal_whole(oracle, kind):
    import ztamd

    text, mixed = corpora(oracle)
    data = mixed
    if kind == "zlib6":
        s = raw(data, 6)
    elif kind == "zlib1":
        s = raw(data, 1, mem=1)  # small blocks (128-symbol buffer)
    elif kind == "zlib9":
        s = raw(text, 9, mem=1)
        data = text
    elif kind == "stored":
        s = raw(data, 0)
    elif kind == "fixed":
        s = raw(data, 6, zlib.Z_FIXED)
    elif kind == "huffman_only":
        s = raw(data, 6, zlib.Z_HUFFMAN_ONLY)
    elif kind == "reference":
        data = text[:200_000]
        s, _ = oracle.raw_deflate(data)
    else:
        s = ztamd.deflate_raw(data, level=6)
    whole, _ = oracle.raw_inflate(s)
    assert whole == data
    rng = random.Random(zlib.crc32(kind.encode()))
    cuts = sorted(set(rng.randrange(1, len(s)) for _ in range(16))) + [len(s)]
    parts, st = stream_in_pieces(s, cuts)
    assert b"".join(parts) == data
    assert st.bfinal
    assert (st.ip * 8 + st.bit + 7) // 8 == len(s)
    if kind not in ("reference",):  # the reference writes one block: it decodes at the end
        assert sum(1 for p in parts if p) >= 2
    # every prefix of the output that was returned is a prefix of the data
    acc = b""
    for p in parts:
        acc += p
        assert data.startswith(acc)


def test_stream_byte_at_a_time(oracle):
    data = oracle.gen("wordsalad", 5, 3000) + oracle.gen("xorshift32", 5, 500)
    c = zlib.compressobj(6, zlib.DEFLATED, -15)
    # many small blocks: flush a block boundary every 400 input bytes
    s = b"".join(c.compress(data[i:i + 400]) + c.flush(zlib.Z_FULL_FLUSH if i % 800 else zlib.Z_SYNC_FLUSH)
                 for i in range(0, len(data), 400)) + c.flush()
    parts, st = stream_in_pieces(s, range(1, len(s) + 1))
    assert b"".join(parts) == data and st.bfinal
    assert sum(1 for p in parts if p) >= 8


def test_stream_window_spans_calls(oracle):
    """Matches that reach back into output returned by earlier calls."""
    chunk = oracle.gen("xorshift32", 9, 20_000)
    data = chunk + oracle.gen("wordsalad", 9, 5000) + chunk  # 25 KB-back repeat
    c = zlib.compressobj(9, zlib.DEFLATED, -15)
    s = c.compress(data[:25_000]) + c.flush(zlib.Z_SYNC_FLUSH) + c.compress(data[25_000:]) + c.flush()
    k = s.index(b"\x00\x00\xff\xff") + 4  # end of the first call's input: the sync flush
    parts, st = stream_in_pieces(s, [k, len(s)])
    assert parts[0] == data[:25_000] and b"".join(parts) == data


def test_truncated_never_raises(oracle):
    import ztamd

    data = oracle.gen("wordsalad", 2, 60_000)
    s = raw(data, 6)
    for end in range(0, len(s), max(1, len(s) // 40)):
        out, end_bits, fin = ztamd.inflate_raw_resume(s[:end])
        assert not fin and data.startswith(out) and end_bits <= 8 * end


def test_corrupt_stream_raises_reference_message():
    import ztamd

    # BTYPE 3 in the first header: src/RawInflate.ts:168
    with pytest.raises(ztamd.ZtError) as e:
        ztamd.RawInflateStream().decompress(b"\x07" + b"\x00" * 64)
    assert e.value.msg == "unknown BTYPE: 3"


def test_resume_at_bit_offset_with_window(oracle):
    """zt_inflate_raw_resume from an unaligned block boundary with the
    preceding output as the window (the state a stream hands over)."""
    import ztamd

    data = oracle.gen("wordsalad", 4, 120_000)
    s = raw(data, 6, mem=2)  # 256-symbol blocks: many unaligned block boundaries
    out1, end1, fin1 = ztamd.inflate_raw_resume(s[: len(s) // 2])
    assert not fin1 and len(out1) > 0
    out2, end2, fin2 = ztamd.inflate_raw_resume(s, end1, out1)
    assert fin2 and out1 + out2 == data
    assert (end2 + 7) // 8 == len(s)


def test_finish_reports_corrupt_tail(oracle):
    """A stream that has fully arrived but is corrupt in its last 8 bytes:
    decompress() keeps waiting for more input (the error is within the last
    64 bits), finish() -- the caller has no more input -- raises the
    stream's own error, as a one-shot decode does.  A truncated stream
    (no final block) raises on finish() too; a valid one finishes."""
    import ztamd

    data = oracle.gen("wordsalad", 21, 200_000)
    good = raw(data)
    st = ztamd.RawInflateStream()
    assert st.finish(good) == data and st.bfinal
    # the whole text, a sync flush, then a final block of BTYPE 3 ("unknown
    # BTYPE: 3", src/RawInflate.ts:168): the error lies in the last 2 bytes
    c = zlib.compressobj(6, zlib.DEFLATED, -15)
    bad = c.compress(data) + c.flush(zlib.Z_SYNC_FLUSH) + b"\x07\x00"
    with pytest.raises(ztamd.ZtError):
        ztamd.inflate_raw(bad)  # the one-shot decode rejects it
    st = ztamd.RawInflateStream()
    st.decompress(bad)
    assert not st.bfinal  # still waiting for input
    with pytest.raises(ztamd.ZtError) as e:
        st.finish()
    assert e.value.msg == "unknown BTYPE: 3"
    st = ztamd.RawInflateStream()
    part = st.decompress(good[: len(good) // 2])
    with pytest.raises(ztamd.ZtError):
        st.finish()
    assert data.startswith(part)
