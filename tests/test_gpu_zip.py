"""Zip / Unzip (csrc/zip_api.cpp) against the reference:
tests/golden/zip.json was written by the reference's own Zip / Unzip
(tools/gen_golden_zip.mjs).  STORE-only archives must be byte-identical to the
reference's; archives with DEFLATE members must have the reference's layout
and header fields with bodies that decode (by the oracle's restated
RawInflate and by zlib) to the inputs.  Unzip must return the reference's
names, data and error messages."""
import hashlib
import zlib

import pytest

from golden_util import blob_bytes, load
from test_zip_fixtures import DATE, gen_spec, parse_zip

pytestmark = pytest.mark.gpu

ZIP = load("zip.json")


@pytest.fixture(scope="module")
def zt():
    import ztamd

    assert ztamd.device_count() > 0, "no GPU visible"
    return ztamd


def _files(zt, oracle, arch):
    mt = zt.dos_mtime(DATE[0], DATE[1] + 1, DATE[2], DATE[3], DATE[4], DATE[5])
    out = []
    for f in arch["files"]:
        o = f["opts"]
        d = dict(data=gen_spec(oracle, f["spec"]), name=f["fn"].encode("latin1"), mtime=mt,
                 method=o.get("compressionMethod", 8), os=o.get("os", 0))
        if "comment" in o:
            d["comment"] = o["comment"].encode("latin1")
        ct = o.get("deflateOptions", {}).get("compressionType")
        if ct is not None:
            d["compression_type"] = ct
        out.append(d)
    return out


@pytest.mark.parametrize("rec", [r for r in ZIP["records"] if r["kind"] == "zip"], ids=lambda r: r["name"])
def test_zip_matches_reference(zt, oracle, rec):
    files = _files(zt, oracle, rec["archive"])
    ours = zt.zip_compress(files, comment=bytes(rec["archive"]["comment"]))
    ref = blob_bytes(rec["output"])
    if all(f["method"] == 0 for f in files):
        assert ours == ref
        return
    a, b = parse_zip(ours), parse_zip(ref)
    assert len(a["entries"]) == len(b["entries"]) == len(files)
    assert a["comment"] == b["comment"]
    for ea, eb, f in zip(a["entries"], b["entries"], files):
        for k in ("name", "comment", "method", "crc32", "plain_size", "mtime", "os", "version", "flags"):
            assert ea[k] == eb[k], k
        body = ours[ea["data_off"]:ea["data_off"] + ea["compressed_size"]]
        if f["method"] == 8:
            out, ip = oracle.raw_inflate(body)
            assert out == f["data"] and ip == len(body)
            assert zlib.decompress(body, -15) == f["data"]
        else:
            assert body == f["data"]
    # and the archive unzips with the engine
    err, ents = zt.unzip(ours, verify=True)
    assert err is None
    assert [e["data"] for e in ents] == [f["data"] for f in files]


def _check_unzip(zt, archive, want, verify):
    err, ents = zt.unzip(archive, verify=verify)
    if not want["ok"]:
        assert err is not None and err.msg == want["error"]["message"]
        return
    assert [e["name"].decode("latin1") for e in ents] == want["names"]
    for e, w in zip(ents, want["files"]):
        if w["ok"]:
            assert e["status"] == 0
            assert len(e["data"]) == w["out"]["len"]
            assert hashlib.sha256(e["data"]).hexdigest() == w["out"]["sha256"]
        else:
            assert e["status"] != 0 and e["message"] == w["error"]["message"]


@pytest.mark.parametrize("rec", ZIP["records"], ids=lambda r: r["kind"] + ":" + r["name"])
@pytest.mark.parametrize("verify", [False, True])
def test_unzip_matches_reference(zt, rec, verify):
    archive = blob_bytes(rec["output"] if rec["kind"] == "zip" else rec["archive"])
    _check_unzip(zt, archive, rec["unzip_verify" if verify else "unzip"], verify)


def test_zip_many_files_roundtrip(zt, oracle):
    """A larger archive (one batch): 300 members of mixed kinds and sizes."""
    import random

    rng = random.Random(7)
    kinds = ["wordsalad", "xorshift32", "structured"]
    files = []
    for i in range(300):
        n = rng.choice([0, 1, 100, 5000, 40000, 200000])
        files.append(dict(data=oracle.gen(kinds[i % 3], i, n) if n else b"", name=f"f{i:03d}".encode(),
                          method=8 if i % 5 else 0, mtime=zt.dos_mtime(2024, 2, 29, 23, 59, 58)))
    arch = zt.zip_compress(files, comment=b"many")
    err, ents = zt.unzip(arch, verify=True)
    assert err is None
    assert [e["data"] for e in ents] == [f["data"] for f in files]
    import io
    import zipfile

    with zipfile.ZipFile(io.BytesIO(arch)) as zf:
        assert zf.testzip() is None
        assert [zf.read(f"f{i:03d}") for i in range(300)] == [f["data"] for f in files]


def test_unzip_data_descriptor(zt, oracle):
    """Archives with data descriptors (general-purpose flag bit 3, local CRC and
    sizes 0 -- what a writer on a non-seekable stream emits): every DEFLATE
    member, including ones far larger than 64 KiB compressed, decodes from
    its offset as the reference's RawInflate would (src/Unzip.ts:284-288).
    The reference itself never returns on such archives (its RawInflate gets
    bufferSize 0, tools/gen_golden_zip.mjs), so this is pinned by Python's
    zipfile, which wrote them."""
    import io
    import zipfile

    class Sink(io.RawIOBase):
        def __init__(self):
            self.buf = bytearray()

        def writable(self):
            return True

        def write(self, b):
            self.buf += b
            return len(b)

    data = [oracle.gen("xorshift32", 31, 300000), oracle.gen("wordsalad", 32, 200000),
            oracle.gen("structured", 33, 150000), b"", b"tail"]
    sink = Sink()
    with zipfile.ZipFile(sink, "w", zipfile.ZIP_DEFLATED) as zf:
        for i, d in enumerate(data):
            zf.writestr(f"m{i}", d)
    arch = bytes(sink.buf)
    entries = parse_zip(arch)["entries"]
    assert all(e["flags"] & 8 for e in entries)
    assert max(e["compressed_size"] for e in entries) > 65536 + 1024
    err, ents = zt.unzip(arch, verify=False)
    assert err is None
    assert [e["data"] for e in ents] == data
