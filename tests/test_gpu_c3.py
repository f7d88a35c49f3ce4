"""Config C3 at full size: RawDeflate level 6 of ONE 8 GiB
device-resident buffer, chunked into 32 KiB blocks, and the sharded layout
of 8(e).  Offsets above 4 GiB are exercised on every kernel of the deflate
and inflate pipelines; the checks are size-independent properties (exact
device round trip) plus oracle decodes of whole 1 MiB segments sampled past
4 GiB (the reference's RawInflate, restated, decodes each segment alone).
Reference: src/RawDeflate.ts:87-114 (one-stream compress), src/RawInflate.ts.
"""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SEG = 1 << 20
MARK = b"\0\0\0\xff\xff\0\0\0\xff\xff"  # restart marker: two empty stored blocks (deflate.hip)


@pytest.fixture(scope="module")
def zt():
    import ztamd

    assert ztamd.device_count() > 0, "no GPU visible"
    return ztamd


def _segment_starts(s):
    """Stream offsets just past each restart marker (a match is skipped whole:
    when the byte before the marker is 00 the pattern also matches one byte
    early, and the start then falls on the marker's second empty block)."""
    out, i = [], s.find(MARK)
    while i >= 0:
        out.append(i + len(MARK))
        i = s.find(MARK, i + len(MARK))
    return out


def test_c3_8gib_roundtrip(zt, oracle):
    import torch

    n = 8 << 30
    d_in = torch.empty(n, dtype=torch.uint8, device="cuda")
    zt.synth_dev("mixed", 11, d_in.data_ptr(), n)
    bound = zt.deflate_bound(n)
    d_c = torch.empty(bound, dtype=torch.uint8, device="cuda")
    dp = zt.DeflatePlan(n, level=6)
    clen = dp.run(d_in.data_ptr(), n, d_c.data_ptr())
    dp.close()
    del dp
    assert 0.3 * n < clen < 0.8 * n
    d_out = torch.empty(n + 4096, dtype=torch.uint8, device="cuda")
    ip_ = zt.InflatePlan(clen, n)
    olen, ip = ip_.run(d_c.data_ptr(), clen, d_out.data_ptr(), d_out.numel())
    ip_.close()
    assert olen == n and ip == clen
    assert torch.equal(d_out[:n], d_in)
    del d_out
    torch.cuda.empty_cache()
    # oracle decodes of whole segments at input offsets past 4 GiB: segment k
    # is the k-th restart interval (1 MiB); its bytes run from the marker
    # before it to the marker after it, and decode alone (no history)
    s = d_c[:clen].cpu().numpy().tobytes()
    starts = [0] + _segment_starts(s)
    assert len(starts) == n // SEG, (len(starts), n // SEG)
    for k in [4096, 4097, 6000, 8191]:  # 4 GiB, just past it, ~5.9 GiB, the last segment
        lo = starts[k]
        hi = starts[k + 1] if k + 1 < len(starts) else clen
        seg = s[lo:hi]
        if k + 1 < len(starts):
            seg += b"\x03\x00"  # close with an empty final fixed block
        out, _ = oracle.raw_inflate(seg)
        want = d_in[k * SEG:(k + 1) * SEG].cpu().numpy().tobytes()
        assert out == want, k


def test_c3_sharded_streams_concatenate(zt, oracle):
    """8(e): segment-aligned shards of one buffer (zt_shard.shard_range),
    each generated in place (zt_synth_dev_at) and deflated alone, concatenate
    into one stream that inflates to the whole buffer."""
    import torch
    from zt_shard import shard_range

    n = (40 << 20) + 12345
    whole = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
    zt.synth_dev("mixed", 11, whole.data_ptr(), n)
    world = 8
    parts = []
    for r in range(world):
        lo, hi = shard_range(n, world, r)
        piece = torch.empty(hi - lo + 64, dtype=torch.uint8, device="cuda")
        zt.synth_dev_at("mixed", 11, lo, piece.data_ptr(), hi - lo)
        assert torch.equal(piece[:hi - lo], whole[lo:hi])
        p = zt.DeflatePlan(hi - lo)
        o = torch.empty(zt.deflate_bound(hi - lo), dtype=torch.uint8, device="cuda")
        c = p.run(piece.data_ptr(), hi - lo, o.data_ptr(), halo=0, final=1 if r == world - 1 else 0)
        torch.cuda.synchronize()
        parts.append(o[:c].cpu().numpy().tobytes())
        p.close()
    s = b"".join(parts)
    g, ip = zt.inflate_raw(s)
    assert ip == len(s)
    assert g == whole[:n].cpu().numpy().tobytes()


def _bench(*args, timeout=600):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], capture_output=True, text=True,
                       timeout=timeout, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


def test_bench_spawns_ranks():
    """bench.py --gpus 2 without a launcher starts two rank processes itself
    (both on this box's GPU when only one is visible) and reports n_gpus 2."""
    line = _bench("--gpus", "2", "--steps", "1", "--warmup", "0", "--size", str(64 << 20))
    assert line["n_gpus"] == 2 and line["scaling"] == "weak"
    assert line["config"]["bytes_total"] == 2 * (64 << 20)


def test_bench_c3_mode_two_ranks():
    line = _bench("--gpus", "2", "--mode", "c3", "--steps", "1", "--warmup", "0", "--size", str((96 << 20) + 4097))
    assert line["n_gpus"] == 2 and line["scaling"] == "strong"
    assert 0.3 < line["ratio"] < 0.8
