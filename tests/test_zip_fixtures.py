"""The Zip / Unzip fixtures the reference wrote (tests/golden/zip.json,
tools/gen_golden_zip.mjs) checked on the CPU with an independent reader
(Python's zipfile): their entries are the generator inputs, so the GPU tests
(tests/test_gpu_zip.py) can rebuild every archive from the record alone."""
import hashlib
import io
import struct
import zipfile

import pytest

from golden_util import blob_bytes, load

ZIP = load("zip.json")
DATE = [2021, 6, 14, 9, 41, 58]  # new Date(2021, 6, 14, 9, 41, 58): July (month index 6)


def gen_spec(oracle, spec):
    if "ascii" in spec:
        return spec["ascii"].encode("latin1")
    return oracle.gen(spec["gen"], spec["seed"], spec["n"])


def dos_mtime(year, month, day, hour, minute, second):
    """src/Zip.ts:130-139 (month 1-12), restated."""
    return bytes([((minute & 7) << 5) | (second >> 1), ((hour << 3) | (minute >> 3)) & 0xFF,
                  ((month & 7) << 5) | day, (((year - 1980) & 0x7F) << 1) | (month >> 3)])


def parse_zip(b):
    """Central directory + local headers (APPNOTE 4.3), for comparisons."""
    eo = b.rfind(b"PK\x05\x06")
    assert eo >= 0
    _, _, _, total, cd_size, cd_off, clen = struct.unpack_from("<HHHHIIH", b, eo + 4)
    out = {"comment": b[eo + 22:eo + 22 + clen], "entries": []}
    p = cd_off
    for _ in range(total):
        assert b[p:p + 4] == b"PK\x01\x02"
        (version, os_, need, flags, method, t, d, crc, csize, usize, nl, xl, cl, _disk, _ia, _ea,
         loff) = struct.unpack_from("<BBHHHHHIIIHHHHHII", b, p + 4)
        name = b[p + 46:p + 46 + nl]
        comment = b[p + 46 + nl + xl:p + 46 + nl + xl + cl]
        assert b[loff:loff + 4] == b"PK\x03\x04"
        lnl, lxl = struct.unpack_from("<HH", b, loff + 26)
        out["entries"].append(dict(version=version, os=os_, need=need, flags=flags, method=method,
                                   mtime=struct.pack("<HH", t, d), crc32=crc, compressed_size=csize,
                                   plain_size=usize, name=name, comment=comment, local_offset=loff,
                                   data_off=loff + 30 + lnl + lxl))
        p += 46 + nl + xl + cl
    return out


@pytest.mark.parametrize("rec", [r for r in ZIP["records"] if r["kind"] == "zip"], ids=lambda r: r["name"])
def test_reference_zip_records(oracle, rec):
    arch = blob_bytes(rec["output"])
    files = rec["archive"]["files"]
    with zipfile.ZipFile(io.BytesIO(arch)) as zf:
        assert [i.filename for i in zf.infolist()] == [f["fn"] for f in files]
        for f in files:
            if f["opts"].get("compressionMethod", 8) in (0, 8):  # zipfile reads STORE / DEFLATE only
                assert zf.read(f["fn"]) == gen_spec(oracle, f["spec"])
    p = parse_zip(arch)
    for e, f in zip(p["entries"], files):
        if f["opts"].get("compressionMethod", 8) not in (0, 8):
            # any other method number: the data stored as-is (src/Zip.ts:92,255)
            assert arch[e["data_off"]:e["data_off"] + e["compressed_size"]] == gen_spec(oracle, f["spec"])
    mt = dos_mtime(DATE[0], DATE[1] + 1, DATE[2], DATE[3], DATE[4], DATE[5])
    for e, f in zip(p["entries"], files):
        assert e["mtime"] == mt
        assert e["method"] == f["opts"].get("compressionMethod", 8)
        assert e["os"] == f["opts"].get("os", 0) and e["version"] == 20
        assert e["crc32"] == oracle.crc32(gen_spec(oracle, f["spec"]))
    assert p["comment"] == bytes(rec["archive"]["comment"])


@pytest.mark.parametrize("rec", ZIP["records"], ids=lambda r: r["kind"] + ":" + r["name"])
def test_unzip_records_consistent(oracle, rec):
    """Where the reference's Unzip succeeded, its outputs are the archive's
    entries as zipfile reads them."""
    arch = blob_bytes(rec["output"] if rec["kind"] == "zip" else rec["archive"])
    u = rec["unzip"]
    if not u["ok"]:
        return
    try:
        zf = zipfile.ZipFile(io.BytesIO(arch))
    except zipfile.BadZipFile:
        return
    with zf:
        methods = {i.filename: i.compress_type for i in zf.infolist()}
        for f in u["files"]:
            if f["ok"] and methods.get(f["name"]) in (0, 8):
                with zf.open(f["name"]) as fh:
                    try:
                        data = fh.read()
                    except zipfile.BadZipFile:
                        continue  # a CRC the reference does not check without verify
                assert hashlib.sha256(data).hexdigest() == f["out"]["sha256"]
