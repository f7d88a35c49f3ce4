"""RawDeflate on the GPU: every stream must be valid RFC 1951 and decode
bit-exactly to its input through the reference's own RawInflate (restated by
the oracle, including its over-strict EOF check), zlib, and the GPU inflate."""
import zlib

import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def zt():
    import ztamd

    assert ztamd.device_count() > 0, "no GPU visible"
    return ztamd


def check_stream(oracle, zt, data, s):
    # reference RawInflate (oracle restatement, src/RawInflate.ts) -- strict EOF semantics included
    out, ip = oracle.raw_inflate(s)
    assert out == data
    assert ip == len(s)
    assert zlib.decompress(s, -15) == data
    g, gip = zt.inflate_raw(s, ref_strict=True)
    assert g == data and gip == len(s)


SIZES = [0, 1, 2, 3, 4, 10, 100, 1000, 4093, 4094, 4095, 4096, 4097, 8191, 32766, 32767, 32768, 32769, 40000,
         65539, 200000]


@pytest.mark.parametrize("kind", ["xorshift32", "wordsalad", "structured"])
@pytest.mark.parametrize("n", SIZES)
def test_roundtrip_sizes(zt, oracle, kind, n):
    d = oracle.gen(kind, 1000 + n, n)
    check_stream(oracle, zt, d, zt.deflate_raw(d))


@pytest.mark.parametrize("ctype", [0, 1, 2])
@pytest.mark.parametrize("level", [1, 4, 6, 9])
def test_options(zt, oracle, ctype, level):
    d = oracle.gen("wordsalad", 5, 150000) + oracle.gen("xorshift32", 5, 50000) + b"\0" * 70000
    s = zt.deflate_raw(d, compression_type=ctype, level=level)
    check_stream(oracle, zt, d, s)
    if ctype == 0:
        assert len(s) == len(d) + 5 * ((len(d) + 65534) // 65535)


def test_special_patterns(zt, oracle):
    pats = [b"\0" * 1000000, b"ab" * 300000, bytes(range(256)) * 4000, b"abcabcabd" * 50000,
            oracle.gen("xorshift32", 3, 100) * 5000]
    for d in pats:
        check_stream(oracle, zt, d, zt.deflate_raw(d))


def test_large_mixed(zt, oracle):
    d = b"".join(oracle.gen(k, 77 + i, 1 << 20) for i, k in enumerate(["wordsalad", "xorshift32", "structured"] * 3))
    s = zt.deflate_raw(d)
    assert zlib.decompress(s, -15) == d
    assert zt.inflate_raw(s)[0] == d


@pytest.mark.parametrize("kind", ["wordsalad", "xorshift32", "structured"])
def test_ratio_vs_reference(zt, oracle, kind):
    """Ratio gate: build bytes / reference bytes <= 1.02
    per generator on 1 MiB windows (the reference is run whole-window, default
    options, via its byte-exact restatement)."""
    d = oracle.gen(kind, 4, 1 << 20)
    ref, _ = oracle.raw_deflate(d)
    ours = zt.deflate_raw(d)
    print(kind, len(ours), len(ref), len(ours) / len(ref))
    assert len(ours) / len(ref) <= 1.02


@pytest.mark.parametrize("offset", [1, 3, 6])
def test_unaligned_device_input(zt, oracle, offset):
    """Device input at an odd byte offset (byte-wise loads in the match and
    cost-based parse kernels) with a partial last block."""
    import torch

    d = oracle.gen("wordsalad", 21, 300001) + b"\0" * 5000 + oracle.gen("structured", 21, 70001)
    t = torch.zeros(len(d) + offset, dtype=torch.uint8, device="cuda")
    t[offset:] = torch.frombuffer(bytearray(d), dtype=torch.uint8).cuda()
    plan = zt.DeflatePlan(len(d))
    out = torch.empty(zt.deflate_bound(len(d)), dtype=torch.uint8, device="cuda")
    n = plan.run(t.data_ptr() + offset, len(d), out.data_ptr())
    torch.cuda.synchronize()
    check_stream(oracle, zt, d, out[:n].cpu().numpy().tobytes())


def test_cost_based_parse_gains(zt, oracle):
    """Levels >= 4 re-parse every block by a shortest-path DP over bit prices
    (optparse_kernel): it must beat the greedy/lazy parse of the same matches."""
    import os

    d = oracle.gen("wordsalad", 8, 1 << 20)
    plain = zt.deflate_raw(d, level=6)
    os.environ["ZT_DF_PARAMS"] = "32,128,1,128,8,16,16,0"  # level 6 match search, no DP
    try:
        greedy = zt.deflate_raw(d, level=6)
    finally:
        del os.environ["ZT_DF_PARAMS"]
    check_stream(oracle, zt, d, plain)
    check_stream(oracle, zt, d, greedy)
    assert len(plain) < 0.97 * len(greedy)


def test_long_runs_cost_parse(zt, oracle):
    """Matches of 258 bytes (the DP's far candidate across its LDS ring wrap)
    mixed with short matches and literals."""
    d = (b"\0" * 3000 + oracle.gen("wordsalad", 4, 700) + b"xy" * 900 + oracle.gen("xorshift32", 4, 300)) * 60
    check_stream(oracle, zt, d, zt.deflate_raw(d, level=9))
    check_stream(oracle, zt, d, zt.deflate_raw(d, level=4))


def test_device_shards_concatenate(zt, oracle):
    """Multi-GPU layout: shards deflated independently (final=0 except the last,
    each primed with a 32 KiB halo) concatenate into one valid stream."""
    import torch

    d = oracle.gen("wordsalad", 9, 3 << 20) + oracle.gen("structured", 9, 1 << 20)
    t = torch.frombuffer(bytearray(d), dtype=torch.uint8).cuda()
    nshard = 4
    per = (len(d) + nshard - 1) // nshard
    per = (per + 32767) // 32768 * 32768
    parts = []
    plan = zt.DeflatePlan(per)
    out = torch.empty(zt.deflate_bound(per), dtype=torch.uint8, device="cuda")
    for k in range(nshard):
        lo, hi = k * per, min(len(d), (k + 1) * per)
        halo = min(lo, 32768)
        n = plan.run(t.data_ptr() + lo, hi - lo, out.data_ptr(), halo=halo, final=1 if hi == len(d) else 0)
        torch.cuda.synchronize()
        parts.append(out[:n].cpu().numpy().tobytes())
    s = b"".join(parts)
    check_stream(oracle, zt, d, s)


def test_segment_parallel_inflate(zt, oracle):
    """Streams longer than one segment (1 MiB) carry restart markers; the
    segment-parallel inflate must give exactly the one-wave result (host and
    device-resident entry points)."""
    import torch

    d = b"".join(oracle.gen(k, 300 + i, (1 << 20) + 12345 * i)
                 for i, k in enumerate(["wordsalad", "structured", "xorshift32", "wordsalad", "structured"]))
    s = zt.deflate_raw(d)
    assert s.count(b"\0\0\0\xff\xff\0\0\0\xff\xff") >= 4
    assert zlib.decompress(s, -15) == d
    out, ip = zt.inflate_raw(s)
    assert out == d and ip == len(s)
    strict, sip = zt.inflate_raw(s, ref_strict=True)  # one-wave path
    assert strict == d and sip == ip
    # device plan
    di = torch.frombuffer(bytearray(s), dtype=torch.uint8).cuda()
    do = torch.empty(len(d) + 100, dtype=torch.uint8, device="cuda")
    p = zt.InflatePlan(len(s), len(d))
    olen, eip = p.run(di.data_ptr(), len(s), do.data_ptr(), do.numel())
    assert olen == len(d) and eip == len(s)
    assert bytes(do[:olen].cpu().numpy()) == d
    # index > 0: the stream starts inside a larger buffer
    pre = b"hdr" * 7
    out2, ip2 = zt.inflate_raw(pre + s, index=len(pre))
    assert out2 == d and ip2 == len(pre) + len(s)


def test_segment_false_candidates(zt, oracle):
    """The restart pattern inside stored data (including exactly at a stored
    block end) must not change the result."""
    pat = b"\0\0\0\xff\xff\0\0\0\xff\xff"
    chunk = bytearray(oracle.gen("xorshift32", 9, 65535))
    chunk[-10:] = pat
    chunk[1000:1010] = pat
    d = bytes(chunk) * 8
    s = zt.deflate_raw(d, compression_type=0)
    assert zt.inflate_raw(s)[0] == d
    # a Huffman stream followed by stored data holding the pattern
    d2 = oracle.gen("wordsalad", 4, 1 << 19) + pat * 40000 + oracle.gen("xorshift32", 4, 1 << 19)
    s2 = zt.deflate_raw(d2)
    zt.release_scratch()
    assert zt.inflate_raw(s2)[0] == d2
    # every false candidate's token slot is bounded by the input bits up to
    # the next candidate: ~80 K candidates must not take a block's slot each
    # (~10 GB); the whole call stays well under 1 GiB of scratch
    dev, _ = zt.scratch_bytes()
    assert dev < (1 << 30), dev
    # a crafted input that is nothing but dense candidates
    junk = pat * 400000
    zt.release_scratch()
    with pytest.raises(zt.ZtError):
        zt.inflate_raw(junk)
    dev, _ = zt.scratch_bytes()
    assert dev < (1 << 30), dev
    # truncated segmented stream: same error as the one-wave decode
    s3 = zt.deflate_raw(oracle.gen("wordsalad", 5, 3 << 20))
    with pytest.raises(zt.ZtError):
        zt.inflate_raw(s3[: len(s3) // 2])


def test_rank_shards_concatenate(zt, oracle):
    """zt_shard layout: segment-aligned shards deflated with halo 0 (final only
    on the last) concatenate into one stream; inflate decodes it
    segment-parallel and exactly."""
    import torch
    from zt_shard import shard_range

    n = 5 * (1 << 20) + 777
    d = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
    zt.synth_dev("mixed", 21, d.data_ptr(), n)
    world = 3
    parts = []
    for r in range(world):
        lo, hi = shard_range(n, world, r)
        p = zt.DeflatePlan(max(1, hi - lo))
        o = torch.empty(zt.deflate_bound(hi - lo), dtype=torch.uint8, device="cuda")
        m = p.run(d.data_ptr() + lo, hi - lo, o.data_ptr(), halo=0, final=1 if r == world - 1 else 0)
        parts.append(bytes(o[:m].cpu().numpy()))
    s = b"".join(parts)
    want = bytes(d[:n].cpu().numpy())
    assert zlib.decompress(s, -15) == want
    out, ip = zt.inflate_raw(s)
    assert out == want and ip == len(s)


def test_two_phase_inflate_is_used(zt, oracle):
    """Our streams carry a sync point after every block: inflate decodes them
    in two phases (tokenize units, resolve segments) and the result equals the
    input; overlapping copies (distance < length) exercise the in-window
    pointer jumping."""
    parts = [oracle.gen("wordsalad", 21, (1 << 20) + 777), b"\0" * (1 << 20) + b"x",
             b"abc" * 400000, oracle.gen("xorshift32", 22, 300001), oracle.gen("structured", 23, 1 << 20),
             bytes(range(256)) * 3000, b"ab" * 70000 + b"q"]
    d = b"".join(parts)
    s = zt.deflate_raw(d)
    zt.timing_enable(True)
    out, ip = zt.inflate_raw(s)
    t = zt.timing_read()
    zt.timing_enable(False)
    assert out == d and ip == len(s)
    assert t["inflate_toks"] == 1, "the two-phase inflate did not run"
    for lvl in (1, 9):
        s = zt.deflate_raw(d, level=lvl)
        out, ip = zt.inflate_raw(s)
        assert out == d and ip == len(s)


@pytest.mark.parametrize("level", [1, 6, 9])
def test_output_does_not_depend_on_the_run(zt, oracle, level):
    """The same input deflates to the same bytes whatever ran on the GPU
    before: the match kernel must not read LDS that no thread of its own
    workgroup wrote (a round-2 bug: the 4-byte table of the first sub-chunk's
    last positions was read uninitialised, so level-1 streams of text
    differed from box to box)."""
    data = oracle.gen("wordsalad", 31, 3 << 20) + oracle.gen("structured", 31, 1 << 20)
    first = zt.deflate_raw(data, level=level)
    for seed in (1, 2):
        # other work leaves other LDS contents behind on every CU
        zt.deflate_raw(oracle.gen("xorshift32", seed, 4 << 20), level=9)
        zt.deflate_raw(oracle.gen("wordsalad", 100 + seed, 4 << 20), level=1)
        assert zt.deflate_raw(data, level=level) == first
    check_stream(oracle, zt, data, first)


@pytest.mark.parametrize("shift", [1, 2, 3])
def test_device_stream_at_unaligned_output(zt, oracle, shift):
    """encode_kernel writes every block straight into the stream at its
    scanned offset, sharing boundary words with its neighbours (byte-masked
    stores): the stream written at d_out + 1 / 2 / 3 equals the aligned one,
    for dynamic, fixed-by-size and stored blocks, restart markers included."""
    import torch

    d = oracle.gen("wordsalad", 31, 5 << 20) + oracle.gen("xorshift32", 31, 1 << 20) + \
        oracle.gen("structured", 31, (3 << 20) + 777)
    n = len(d)
    d_in = torch.frombuffer(bytearray(d), dtype=torch.uint8).cuda()
    dp = zt.DeflatePlan(n, level=6)
    d_a = torch.zeros(zt.deflate_bound(n) + 16, dtype=torch.uint8, device="cuda")
    la = dp.run(d_in.data_ptr(), n, d_a.data_ptr())
    d_u = torch.full((zt.deflate_bound(n) + 16,), 0xA5, dtype=torch.uint8, device="cuda")
    lu = dp.run(d_in.data_ptr(), n, d_u.data_ptr() + shift)
    dp.close()
    torch.cuda.synchronize()
    a = d_a[:la].cpu().numpy().tobytes()
    u = d_u.cpu().numpy().tobytes()
    assert la == lu and u[shift:shift + lu] == a
    assert u[:shift] == b"\xa5" * shift and u[shift + lu] == 0xA5  # neighbours untouched
    assert zlib.decompress(a, -15) == d


def _plan_inflate(zt, s, cap):
    import torch

    di = torch.frombuffer(bytearray(s), dtype=torch.uint8).cuda()
    do = torch.full((cap + 64,), 0x5A, dtype=torch.uint8, device="cuda")
    p = zt.InflatePlan(len(s), cap)
    try:
        olen, eip = p.run(di.data_ptr(), len(s), do.data_ptr(), cap)
    finally:
        p.close()
    torch.cuda.synchronize()
    return olen, eip, do.cpu().numpy().tobytes()


def test_device_chain(zt, oracle):
    """zt_inflate_dev into a caller's buffer builds the unit chain, the copy
    segments and their descriptor offsets on the device (chain_kernel) when
    every unit follows the one before -- text, stored runs (classify_kernel's
    random windows: direct segments), restart markers, ragged end -- and the
    bytes past the output stay untouched."""
    d = b"".join([oracle.gen("wordsalad", 41, (3 << 20) + 5), oracle.gen("xorshift32", 41, (2 << 20) + 3),
                  oracle.gen("structured", 41, (1 << 20) + 1), b"\0" * 70001, oracle.gen("wordsalad", 42, 12345)])
    s = zt.deflate_raw(d)
    zt.timing_enable(True)
    olen, eip, out = _plan_inflate(zt, s, len(d) + 1000)
    t = zt.timing_read()
    zt.timing_enable(False)
    assert t["inflate_toks"] == 1, "the two-phase inflate did not run"
    assert olen == len(d) and eip == len(s)
    assert out[:olen] == d and out[olen:olen + 64] == b"\x5a" * 64
    # the same stream through the host API (host-built chain)
    assert zt.inflate_raw(s) == (d, len(s))


def test_device_chain_falls_back(zt, oracle):
    """Streams the device chain does not take -- false sync-point candidates
    inside stored data, an output capacity below the stream's size -- give
    the host walk's results."""
    pat = b"\0\0\0\xff\xff\0\0\0\xff\xff"
    d = oracle.gen("wordsalad", 4, 1 << 19) + pat * 40000 + oracle.gen("xorshift32", 4, 1 << 19)
    s = zt.deflate_raw(d)
    olen, eip, out = _plan_inflate(zt, s, len(d) + 100)
    assert olen == len(d) and eip == len(s) and out[:olen] == d
    chunk = bytearray(oracle.gen("xorshift32", 9, 65535))
    chunk[-10:] = pat
    chunk[1000:1010] = pat
    d2 = bytes(chunk) * 8
    s2 = zt.deflate_raw(d2, compression_type=0)
    olen, eip, out = _plan_inflate(zt, s2, len(d2))
    assert olen == len(d2) and out[:olen] == d2
    # capacity one byte short
    d3 = oracle.gen("wordsalad", 5, 3 << 20)
    s3 = zt.deflate_raw(d3)
    with pytest.raises(zt.ZtError):
        _plan_inflate(zt, s3, len(d3) - 1)
    olen, eip, out = _plan_inflate(zt, s3, len(d3))
    assert olen == len(d3) and out[:olen] == d3


def test_tail_split_streams_identical(zt, oracle):
    """The match kernel's last round of workgroups takes one block each
    (deflate_geometry: ZT_DF_TAILK) instead of the super-chunk's four: every
    position is linked and searched alike whatever workgroup holds it, so the
    stream of an input large enough to have a tail round (48 MiB: 1536 blocks,
    1024 of them in one-block workgroups on 256 CUs) is byte-identical to the
    one without the split (a child process with ZT_DF_TAILK=0), and decodes."""
    import hashlib
    import json
    import os
    import subprocess
    import sys

    import torch

    n = 48 << 20
    d_in = torch.empty(n, dtype=torch.uint8, device="cuda")
    d_c = torch.empty(zt.deflate_bound(n), dtype=torch.uint8, device="cuda")
    zt.synth_dev("mixed", 7, d_in.data_ptr(), n)
    dp = zt.DeflatePlan(n, level=6)
    clen = dp.run(d_in.data_ptr(), n, d_c.data_ptr())
    dp.close()
    torch.cuda.synchronize()
    s = d_c[:clen].cpu().numpy().tobytes()
    assert zlib.decompress(s, -15) == d_in.cpu().numpy().tobytes()
    here = os.path.dirname(os.path.abspath(__file__))
    env = dict(os.environ, ZT_DF_TAILK="0")
    p = subprocess.run([sys.executable, os.path.join(here, "tail_split_child.py")], env=env, capture_output=True,
                       text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-2000:]
    child = json.loads(p.stdout.strip().splitlines()[-1])
    assert child == {"len": clen, "sha256": hashlib.sha256(s).hexdigest()}
