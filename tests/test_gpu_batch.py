"""Batch compression (csrc/batch_api.cpp, config C4): many independent
buffers in one pipeline per device.  Every GZip member is checked against the
single-buffer call's header, decoded bit-exactly by the oracle's RawInflate
(the reference's algorithm restated, pinned by tests/golden) and by the
engine's GUnzip, with the oracle's CRC-32 / Adler-32 in the trailers."""
import math
import random
import zlib

import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def zt():
    import ztamd

    assert ztamd.device_count() > 0, "no GPU visible"
    return ztamd


def _files(oracle, count, seed, lo=1 << 10, hi=1 << 20):
    """SURVEY 8(d) C4's size distribution (log-uniform 1 KiB - 1 MiB), mixed
    text / binary, plus the edge sizes the batch path must handle."""
    rng = random.Random(seed)
    kinds = ["wordsalad", "xorshift32", "structured"]
    out = [b"", b"x", bytes(range(256)) * 128, b"\0" * 32768, b"\0" * 32769]
    while len(out) < count:
        n = int(math.exp(rng.uniform(math.log(lo), math.log(hi))))
        out.append(oracle.gen(kinds[len(out) % 3], seed * 7919 + len(out), n))
    return out


def test_gzip_batch_members(zt, oracle):
    files = _files(oracle, 160, 1)
    members = zt.gzip_compress_batch(files)
    head = oracle.gzip_header()
    assert len(members) == len(files)
    for f, m in zip(files, members):
        assert m[:len(head)] == head
        body_out, ip = oracle.raw_inflate(m, index=len(head))
        assert body_out == f
        assert m[ip:ip + 4] == oracle.crc32(f).to_bytes(4, "little")
        assert m[ip + 4:] == (len(f) & 0xFFFFFFFF).to_bytes(4, "little")
    # the engine's GUnzip over the concatenated members (multi-member file)
    cat = b"".join(members[:40])
    out, mem = zt.gunzip(cat)
    assert out == b"".join(files[:40]) and len(mem) == 40


def test_gzip_batch_opts_match_single(zt, oracle):
    files = _files(oracle, 24, 2, hi=200 << 10)
    kw = dict(name=b"file.txt", comment=b"batch", hcrc=True, mtime=1234567)
    members = zt.gzip_compress_batch(files, **kw)
    for f, m in zip(files, members):
        single, crc = zt.gzip_compress(f, **kw)
        h = oracle.gzip_header(name=b"file.txt", comment=b"batch", hcrc=True, mtime=1234567)
        assert m[:len(h)] == single[:len(h)] == h
        assert m[-8:] == single[-8:]
        assert zlib.decompress(m, 31) == f


@pytest.mark.parametrize("level", [1, 6, 9])
def test_deflate_raw_batch(zt, oracle, level):
    files = _files(oracle, 64, 3 + level, hi=400 << 10)
    streams = zt.deflate_raw_batch(files, level=level)
    for f, s in zip(files, streams):
        out, ip = oracle.raw_inflate(s)
        assert out == f and ip == len(s)


def test_deflate_raw_batch_types(zt, oracle):
    files = _files(oracle, 20, 9, hi=150 << 10)
    for ct in (0, 1):
        streams = zt.deflate_raw_batch(files, compression_type=ct)
        for f, s in zip(files, streams):
            assert oracle.raw_inflate(s)[0] == f


def test_zlib_batch(zt, oracle):
    files = _files(oracle, 48, 4, hi=300 << 10)
    streams = zt.zlib_compress_batch(files)
    for f, s in zip(files, streams):
        assert s[:2] == oracle.zlib_header()
        assert zlib.decompress(s) == f
        assert int.from_bytes(s[-4:], "big") == oracle.adler32(f)


def test_batch_ratio_matches_single(zt, oracle):
    """Batch streams compress like the one-buffer call (history never crosses
    buffers, so a buffer's stream depends only on its own bytes)."""
    files = _files(oracle, 12, 5, lo=40 << 10, hi=300 << 10)
    b = zt.deflate_raw_batch(files)
    for f, s in zip(files, b):
        one = zt.deflate_raw(f)
        assert abs(len(s) - len(one)) <= max(64, len(one) // 50)


def test_set_devices(zt, oracle):
    n = zt.device_count()
    files = _files(oracle, 30, 6, hi=128 << 10)
    zt.set_devices((1 << n) - 1)
    try:
        members = zt.gzip_compress_batch(files)
    finally:
        zt.set_devices(0)
    for f, m in zip(files, members):
        assert zlib.decompress(m, 31) == f
    with pytest.raises(zt.ZtError):
        zt.set_devices(1 << n)


@pytest.mark.parametrize("kind", ["gzip", "zlib"])
def test_grouped_batch_equals_single_pipeline(zt, kind):
    """A batch of >= 256 MiB runs as a grouped three-stage pipeline
    (batch_api.cpp batch_grouped); every member must equal the one the single
    pipeline writes for the same file (two halves of the batch, each below
    the threshold) and decode to its input (Python zlib, independent)."""
    import random
    import zlib

    import torch

    rng = random.Random(5)
    sizes = []
    while sum(sizes) < (300 << 20):
        sizes.append(int(2 ** rng.uniform(10, 21)) + rng.randrange(7))
    total = sum(sizes)
    d = torch.empty(total, dtype=torch.uint8, device="cuda")
    zt.synth_dev("mixed", 9, d.data_ptr(), total)
    host = d.cpu().numpy().tobytes()
    files, o = [], 0
    for s in sizes:
        files.append(host[o:o + s])
        o += s
    fn = zt.gzip_compress_batch if kind == "gzip" else zt.zlib_compress_batch
    whole = fn(files)
    half = len(files) // 2
    parts = fn(files[:half]) + fn(files[half:])
    assert len(whole) == len(files)
    assert whole == parts
    for f, mb in zip(files[::97], whole[::97]):
        dec = zlib.decompress(mb, 31 if kind == "gzip" else 15)
        assert dec == f


@pytest.mark.parametrize("ndev", [2, 3])
def test_alias_devices_split(ndev):
    """The multi-device batch split (zt_set_devices: LPT over the devices, one
    host thread and one context per device, batch_api.cpp run_batch) run on
    this one GPU: ZT_ALIAS_DEVICES makes the library present `ndev` logical
    devices, each with its own context.  Every member spread over them equals
    the one-device member and decodes with the oracle (tests/alias_batch_child.py,
    a child process: the alias is read once when the library loads)."""
    import json
    import os
    import subprocess
    import sys

    here = os.path.dirname(os.path.abspath(__file__))
    env = dict(os.environ, ZT_ALIAS_DEVICES=str(ndev))
    p = subprocess.run([sys.executable, os.path.join(here, "alias_batch_child.py"), str(ndev)], env=env,
                       capture_output=True, text=True, timeout=100)
    assert p.returncode == 0, p.stderr[-2000:]
    res = json.loads(p.stdout.strip().splitlines()[-1])
    assert res == {"logical_devices": ndev, "gzip_equal": True, "raw_equal": True, "oracle_ok": True,
                   "crc_ok": True}, res
