"""Pin the CPU oracle (oracle/zt_oracle.c) against vectors produced by the
reference's own JS (tools/gen_golden.mjs).  CPU only."""
import pytest

from golden_util import blob_matches, load, make_input
from zt_oracle import OracleError

CK = load("checksums.json")
DF = load("deflate.json")
INF = load("inflate.json")


@pytest.mark.parametrize("rec", CK["records"], ids=lambda r: str(r["input"])[:48])
def test_checksums(oracle, rec):
    d = make_input(rec["input"], oracle)
    assert oracle.crc32(d) == rec["crc32"]
    assert oracle.adler32(d) == rec["adler32"]
    if "crc32_chain" in rec:
        cut = len(d) >> 1
        assert oracle.crc32(d[cut:], oracle.crc32(d[:cut])) == rec["crc32_chain"]
        assert oracle.adler32(d[cut:], oracle.adler32(d[:cut])) == rec["adler32_chain"]
    if "crc32_pos3" in rec:
        # src/CRC32.ts:27 -- length defaults to data.length even with pos>0: the
        # 3 bytes read past the end are `undefined`, i.e. XORed as 0
        assert oracle.crc32(d[3:] + b"\0\0\0") == rec["crc32_pos3"]
    if "adler32_len_pos" in rec:
        assert oracle.adler32(d[2:2 + len(d) - 5], 7) == rec["adler32_len_pos"]


def test_survey_pins(oracle):
    # SURVEY.md 8(c) pins
    assert oracle.crc32(b"123456789") == 0xCBF43926
    assert oracle.adler32(b"123456789") == 0x091E01DE
    d = oracle.gen("xorshift32", 1, 65536)
    assert oracle.crc32(d) == 0x9F2BA2F0 and oracle.adler32(d) == 0x17126908
    assert oracle.raw_deflate(b"")[0].hex() == "05c0810800000000207feb03"
    assert oracle.raw_deflate(b"AAA")[0].hex() == "05c081080000000020b6fda50e01"


@pytest.mark.parametrize("rec", CK["singles"], ids=lambda r: f"{r['num']}-{r['crc']}")
def test_crc32_single(oracle, rec):
    out = oracle.crc32_single(rec["num"], rec["crc"])
    # the reference returns an Int32 (no >>> 0)
    if out >= 1 << 31:
        out -= 1 << 32
    assert out == rec["out"]


@pytest.mark.parametrize("rec", CK["strings"], ids=lambda r: repr(r["str"]))
def test_adler32_strings(oracle, rec):
    # src/Util.ts:5-12 stringToByteArray: charCode & 0xFF
    b = bytes(ord(c) & 0xFF for c in rec["str"])
    assert oracle.adler32(b) == rec["adler32"]


def _deflate_id(r):
    return f"{str(r['input'])[:40]}|{r['opts']}"


@pytest.mark.parametrize("rec", DF["records"], ids=_deflate_id)
def test_raw_deflate(oracle, rec):
    d = make_input(rec["input"], oracle)
    o = rec["opts"]
    ob = bytes.fromhex(o["outputBuffer"]) if "outputBuffer" in o else None
    kw = dict(lazy=o.get("lazy", 0), ctype=o.get("compressionType", 2), outbuf=ob, out_index=o.get("outputIndex", 0))
    if "error" in rec:
        with pytest.raises(OracleError):
            oracle.raw_deflate(d, **kw)
        return
    out, op = oracle.raw_deflate(d, **kw)
    assert op == rec["op"]
    assert blob_matches(rec["out"], out)


def _inflate_id(r):
    return f"{str(r['origin'])[:60]}|{r['opts']}"


@pytest.mark.parametrize("rec", INF["records"], ids=_inflate_id)
def test_raw_inflate(oracle, rec):
    from golden_util import blob_bytes

    s = blob_bytes(rec["stream"])
    o = rec["opts"]
    kw = dict(index=o.get("index", 0), buffer_type=o.get("bufferType", 1), buffer_size=o.get("bufferSize", 0x8000))
    if "error" in rec:
        with pytest.raises(OracleError) as ei:
            oracle.raw_inflate(s, **kw)
        assert ei.value.msg == rec["error"]
        return
    out, ip = oracle.raw_inflate(s, **kw)
    assert ip == rec["ip"]
    assert blob_matches(rec["out"], out)


def test_deflate_records_roundtrip_flags(oracle):
    """The reference's own inflate rejects some of its own valid streams
    (over-strict EOF check, src/RawInflate.ts:187); the oracle reproduces the
    exact error on each of them."""
    seen = 0
    for rec in DF["records"]:
        if "inflate_error" not in rec or "hex" not in rec.get("out", {}):
            continue
        s = bytes.fromhex(rec["out"]["hex"])
        with pytest.raises(OracleError) as ei:
            oracle.raw_inflate(s)
        assert ei.value.msg == rec["inflate_error"]
        seen += 1
    assert seen > 10
