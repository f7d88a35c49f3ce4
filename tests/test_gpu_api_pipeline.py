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
