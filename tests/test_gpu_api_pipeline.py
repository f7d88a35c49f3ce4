"""zt_deflate_raw on large host buffers: the input crosses PCIe in
restart-aligned pieces while earlier pieces are deflated and their streams
come back (deflate_api.cpp deflate_raw_pipelined).  The pipelined call must
write exactly the stream a single device-resident deflate of the whole
buffer writes, and that stream must round-trip.  Sizes cover the threshold
(64 MiB), a one-byte last piece and a piece count that is not a power of two.
Reference: src/RawDeflate.ts:87-114 (one call, one stream).
"""
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def zt():
    import ztamd

    assert ztamd.device_count() > 0, "no GPU visible"
    return ztamd


def _device_stream(zt, torch, d_in, n, level):
    d_c = torch.empty(zt.deflate_bound(n), dtype=torch.uint8, device="cuda")
    dp = zt.DeflatePlan(n, level=level)
    clen = dp.run(d_in.data_ptr(), n, d_c.data_ptr())
    dp.close()
    return d_c[:clen].cpu().numpy().tobytes()


@pytest.mark.parametrize("n,level,kind", [
    ((64 << 20) + 1, 6, "mixed"),          # 3 pieces of 32 MiB, the last one byte
    ((160 << 20) + 12345, 6, "mixed"),     # 6 pieces, ragged last one
    (300 << 20, 1, "wordsalad"),           # 8 pieces of 38 MiB (rounded up to 1 MiB segments)
])
def test_pipelined_deflate_equals_single_call(zt, n, level, kind):
    import numpy as np
    import torch

    d_in = torch.empty(n, dtype=torch.uint8, device="cuda")
    zt.synth_dev(kind, 7, d_in.data_ptr(), n)
    host = d_in.cpu().numpy()
    s_host = zt.deflate_raw(memoryview(host), level=level)
    s_dev = _device_stream(zt, torch, d_in, n, level)
    assert len(s_host) == len(s_dev)
    assert s_host == s_dev
    back, ip = zt.inflate_raw(s_host)
    assert ip == len(s_host) and len(back) == n
    assert np.array_equal(np.frombuffer(back, dtype=np.uint8), host)


def test_pipelined_fixed_codes(zt):
    """compressionType FIXED takes the same pipeline (BFINAL on the last piece only)."""
    import numpy as np
    import torch

    n = (96 << 20) + 777
    d_in = torch.empty(n, dtype=torch.uint8, device="cuda")
    zt.synth_dev("structured", 3, d_in.data_ptr(), n)
    host = d_in.cpu().numpy()
    s = zt.deflate_raw(memoryview(host), compression_type=1)
    back, ip = zt.inflate_raw(s)
    assert ip == len(s) and np.array_equal(np.frombuffer(back, dtype=np.uint8), host)


# ---- zt_inflate_raw: the same three-stage pipeline for inflate ----
# (inflate_api.cpp inflate_raw_pipelined: the input is cut after restart
# markers, each non-final piece decoded as a stream of its own with an empty
# final stored block appended on the device; any piece that does not end
# exactly there sends the whole stream to the one-call decode)

def _device_inflate(zt, torch, s, n_out):
    d_s = torch.frombuffer(bytearray(s), dtype=torch.uint8).cuda()
    d_o = torch.empty(n_out + 64, dtype=torch.uint8, device="cuda")
    ip_ = zt.InflatePlan(len(s), n_out + 64)
    ol, ip = ip_.run(d_s.data_ptr(), len(s), d_o.data_ptr(), n_out + 64)
    ip_.close()
    return d_o[:ol].cpu().numpy().tobytes(), ip


@pytest.mark.parametrize("n,kind,tail", [
    ((96 << 20) + 5, "mixed", b""),                 # ~6 pieces of 8 MiB of stream
    ((224 << 20) + 4099, "wordsalad", b""),         # pieces of 8-32 MiB, ragged last
    ((160 << 20) + 17, "structured", b"\x07" * 33),  # trailing bytes after the stream
])
def test_pipelined_inflate_equals_single_call(zt, n, kind, tail):
    import numpy as np
    import torch

    d_in = torch.empty(n, dtype=torch.uint8, device="cuda")
    zt.synth_dev(kind, 9, d_in.data_ptr(), n)
    host = d_in.cpu().numpy()
    s = _device_stream(zt, torch, d_in, n, 6)
    assert len(s) >= 32 << 20  # (the pipelined path's threshold)
    back, ip = zt.inflate_raw(s + tail)
    assert ip == len(s) and len(back) == n
    assert np.array_equal(np.frombuffer(back, dtype=np.uint8), host)
    dev, dip = _device_inflate(zt, torch, s + tail, n)
    assert dip == ip and dev == back


def test_pipelined_inflate_false_markers_in_stored_data(zt):
    """The restart-marker bytes inside stored payloads (compressionType NONE):
    every cut there fails its piece check and the one-call decode runs."""
    import zlib

    rng = __import__("random").Random(3)
    marker = bytes([0, 0, 0, 0xFF, 0xFF, 0, 0, 0, 0xFF, 0xFF])
    parts = []
    for i in range(48):
        parts.append(rng.randbytes(1 << 20))
        parts.append(marker)
    data = b"".join(parts)
    s = zt.deflate_raw(data, compression_type=0)
    back, ip = zt.inflate_raw(s)
    assert ip == len(s) and back == data
    assert zlib.decompress(s, -15) == data


def test_pipelined_inflate_zlib_stream(zt):
    """A foreign stream (zlib level 1, no restart markers) is decoded in one call."""
    import zlib

    import torch

    n = 80 << 20
    d_in = torch.empty(n, dtype=torch.uint8, device="cuda")
    zt.synth_dev("wordsalad", 4, d_in.data_ptr(), n)
    data = d_in.cpu().numpy().tobytes()
    co = zlib.compressobj(1, zlib.DEFLATED, -15)
    s = co.compress(data) + co.flush()
    back, ip = zt.inflate_raw(s)
    assert ip == len(s) and back == data
