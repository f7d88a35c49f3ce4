"""zt_deflate_raw on large host buffers: the input crosses PCIe in
restart-aligned pieces while earlier pieces are deflated and their streams
come back (deflate_api.cpp deflate_raw_pipelined).  The pipelined call must
write exactly the stream a single device-resident deflate of the whole
buffer writes, and that stream must round-trip.  Sizes cover the threshold
(64 MiB), a one-byte last piece, a piece count that is not a power of two and
the growing pieces of inputs from 512 MiB.
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
    ((576 << 20) + 333, 6, "mixed"),       # the ramp from 512 MiB: 64, 128, 256, 128 MiB and 333 bytes
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


# ---- the host output pool (zt_api.cpp host_out): zt_free hands large outputs
# back, the next output of a similar size reuses the buffer registered with
# HIP, and copies to / from it go by DMA without staging.  The bench's host
# round trip exactly: deflate output pointer straight into zt_inflate_raw.

def test_host_output_pool_round_trips(zt):
    import ctypes

    import numpy as np
    import torch

    n = (96 << 20) + 4097
    d_in = torch.empty(n, dtype=torch.uint8, device="cuda")
    zt.synth_dev("mixed", 21, d_in.data_ptr(), n)
    host = d_in.cpu().numpy()
    src = host.ctypes.data_as(ctypes.c_void_p)
    opts = zt.DeflateOpts(2, 0, 6)
    iopts = zt.InflateOpts(1, 0x8000, 0)
    first = None
    held = []
    for rep in range(4):
        out = ctypes.POINTER(ctypes.c_uint8)()
        olen = ctypes.c_size_t()
        zt._check(zt.lib.zt_deflate_raw(src, n, ctypes.byref(opts), ctypes.byref(out), ctypes.byref(olen)))
        s = ctypes.string_at(out, olen.value)
        first = s if first is None else first
        assert s == first  # the same stream from a fresh and from a reused (registered) buffer
        back = ctypes.POINTER(ctypes.c_uint8)()
        blen, ip = ctypes.c_size_t(), ctypes.c_size_t()
        zt._check(zt.lib.zt_inflate_raw(out, olen.value, 0, ctypes.byref(iopts), ctypes.byref(back),
                                        ctypes.byref(blen), ctypes.byref(ip)))
        assert blen.value == n and ip.value == olen.value
        assert np.array_equal(np.ctypeslib.as_array(back, shape=(n,)), host)
        zt.lib.zt_free(out)
        if rep == 1:
            held.append(back)  # kept alive: the next outputs must not reuse it
        else:
            zt.lib.zt_free(back)
    assert np.array_equal(np.ctypeslib.as_array(held[0], shape=(n,)), host)
    zt.lib.zt_free(held[0])


# ---- round 6: the pipelined inflate at any output ratio, and its error paths
# (the output was sized 4x the input and a piece past it sent the
# whole stream to the one-call decode; a failing pipeline returned its output
# buffer while copies into it could still be running)

def _pieces_decoded(zt, fn):
    """Run fn() and return how many decodes the segment path made (the
    pipelined call makes one per piece; the one-call decode makes one)."""
    zt.timing_enable(True)
    r = fn()
    paths = zt.timing_read()["inflate_paths"]
    zt.timing_enable(False)
    return r, paths[0]


def test_pipelined_inflate_high_ratio_stays_pipelined(zt):
    """wordsalad at level 6 compresses ~6.5:1: every piece stays in the
    pipeline (no second decode of the whole stream), output exact."""
    import numpy as np
    import torch

    n = 256 << 20
    d_in = torch.empty(n, dtype=torch.uint8, device="cuda")
    zt.synth_dev("wordsalad", 12, d_in.data_ptr(), n)
    host = d_in.cpu().numpy()
    s = _device_stream(zt, torch, d_in, n, 6)
    assert len(s) >= 32 << 20 and n > 4 * len(s)
    (back, ip), decodes = _pieces_decoded(zt, lambda: zt.inflate_raw(s))
    assert ip == len(s) and len(back) == n
    assert np.array_equal(np.frombuffer(back, dtype=np.uint8), host)
    assert decodes >= 2, "the stream left the pipeline"


def test_pipelined_inflate_ratio_jump_grows_outputs(zt):
    """Piece 0 is incompressible (ratio 1) and the last piece holds 192 MiB
    of one repeated byte: its device slot and the host output both grow
    (one more decode of that piece, one move of the bytes so far) and the
    result equals the data."""
    import numpy as np
    import torch

    a, z = 40 << 20, 192 << 20
    d_in = torch.empty(a + z, dtype=torch.uint8, device="cuda")
    zt.synth_dev("xorshift32", 5, d_in.data_ptr(), a)
    d_in[a:] = 0x61
    host = d_in.cpu().numpy()
    s = _device_stream(zt, torch, d_in, a + z, 6)
    assert len(s) >= 32 << 20
    (back, ip), decodes = _pieces_decoded(zt, lambda: zt.inflate_raw(s))
    assert ip == len(s) and len(back) == a + z
    assert np.array_equal(np.frombuffer(back, dtype=np.uint8), host)
    assert decodes >= 2, "the stream left the pipeline"


def test_pipelined_inflate_failure_on_registered_output(zt):
    """A pipelined inflate that fails in its last piece after earlier pieces
    were copied straight into a registered pool buffer: the call returns the
    stream's error (or its one-call result) only after every copy finished,
    and the pool stays usable -- the good stream decodes exactly afterwards."""
    import ctypes

    import numpy as np
    import torch

    n = 192 << 20
    d_in = torch.empty(n, dtype=torch.uint8, device="cuda")
    zt.synth_dev("mixed", 31, d_in.data_ptr(), n)
    host = d_in.cpu().numpy()
    s = _device_stream(zt, torch, d_in, n, 6)
    iopts = zt.InflateOpts(1, 0x8000, 0)

    def inflate(buf):
        arr = np.frombuffer(buf, dtype=np.uint8)
        back = ctypes.POINTER(ctypes.c_uint8)()
        blen, ip = ctypes.c_size_t(), ctypes.c_size_t()
        rc = zt.lib.zt_inflate_raw(arr.ctypes.data_as(ctypes.c_void_p), len(buf), 0, ctypes.byref(iopts),
                                   ctypes.byref(back), ctypes.byref(blen), ctypes.byref(ip))
        out = np.ctypeslib.as_array(back, shape=(blen.value,)).copy() if rc == 0 else None
        if rc == 0:
            zt.lib.zt_free(back)
        return rc, out

    for _ in range(2):  # the second output comes from the (now registered) pool
        rc, out = inflate(s)
        assert rc == 0 and np.array_equal(out, host)
    bad = bytearray(s)
    bad[-(256 << 10):-64] = b"\xff" * ((256 << 10) - 64)  # the last piece's blocks: broken
    for _ in range(3):
        rc, out = inflate(bytes(bad))
        assert rc != 0 or len(out) != n or not np.array_equal(out, host)
    rc, out = inflate(s)
    assert rc == 0 and np.array_equal(out, host)
