"""The oracle's container restatement (tests/zt_oracle.py: GUnzip, Inflate,
GZip/Deflate headers) checked against every record the REFERENCE produced in
tests/golden/containers.json (tools/gen_golden_containers.mjs).  CPU only."""
import pytest

from golden_util import blob_bytes, blob_matches, load, make_input
from zt_oracle import OracleError

REC = load("containers.json")["records"]


def _id(r):
    return f"{r['kind']}|{r.get('name') or r.get('input')}|{r.get('opts', r.get('compressionType'))}"


def check_gunzip(oracle, stream, want):
    if not want["ok"]:
        with pytest.raises(OracleError) as ei:
            oracle.gunzip(stream)
        assert ei.value.msg == want["error"]["message"]
        return
    out, members = oracle.gunzip(stream)
    assert blob_matches(want["out"], out)
    assert want["crc32"] == members[-1]["crc32"]
    assert len(members) == len(want["members"])
    for m, w in zip(members, want["members"]):
        assert (m["flg"], m["xfl"], m["os"], m["mtime"]) == (w["flg"], w["xfl"], w["os"], w["mtime"])
        for k in ("name", "comment"):
            assert (None if m[k] is None else m[k].decode("latin1")) == w[k]
        assert blob_matches(w["data"], m["data"])


@pytest.mark.parametrize("rec", [r for r in REC if r["kind"] == "gzip"], ids=_id)
def test_gzip_records(oracle, rec):
    """Header bytes (mtime aside) are the oracle's; GUnzip of the reference's
    member is the oracle's."""
    data = make_input(rec["input"], oracle)
    out = blob_bytes(rec["output"])
    o = rec["opts"]
    name = oracle.header_bytes(o["filename"]) if o.get("filename") else None
    comment = oracle.header_bytes(o["comment"]) if o.get("comment") else None
    mtime = int.from_bytes(out[4:8], "little")
    hd = oracle.gzip_header(name, comment, bool(o.get("hcrc")), mtime)
    assert out[:len(hd)] == hd
    assert rec["crc32"] == oracle.crc32(data)
    if rec["gunzip"]["ok"]:
        assert out[-8:] == oracle.crc32(data).to_bytes(4, "little") + len(data).to_bytes(4, "little")
    check_gunzip(oracle, out, rec["gunzip"])


@pytest.mark.parametrize("rec", [r for r in REC if r["kind"] == "gunzip"], ids=_id)
def test_gunzip_records(oracle, rec):
    check_gunzip(oracle, blob_bytes(rec["stream"]), rec["gunzip"])


@pytest.mark.parametrize("rec", [r for r in REC if r["kind"] == "zlib" and "output" in r], ids=_id)
def test_zlib_records(oracle, rec):
    data = make_input(rec["input"], oracle)
    out = blob_bytes(rec["output"])
    assert out[:2] == oracle.zlib_header(rec["compressionType"])
    assert rec["adler32"] == oracle.adler32(data)
    for verify in (False, True):
        want = rec[f"inflate_{str(verify).lower()}"]
        if not want["ok"]:
            with pytest.raises(OracleError) as ei:
                oracle.zlib_inflate(out, verify=verify)
            assert ei.value.msg == want["error"]["message"]
            continue
        back, ip = oracle.zlib_inflate(out, verify=verify)
        assert blob_matches(want["out"], back) and ip == want["ip"]
        assert back == data


@pytest.mark.parametrize("rec", [r for r in REC if r["kind"] == "inflate"], ids=_id)
def test_inflate_records(oracle, rec):
    s = blob_bytes(rec["stream"])
    o = rec["opts"]
    want = rec["inflate"]
    if not want["ok"]:
        with pytest.raises(OracleError) as ei:
            oracle.zlib_inflate(s, index=o.get("index", 0), verify=o.get("verify", False))
        assert ei.value.msg == want["error"]["message"]
        return
    back, ip = oracle.zlib_inflate(s, index=o.get("index", 0), verify=o.get("verify", False))
    assert blob_matches(want["out"], back) and ip == want["ip"]
