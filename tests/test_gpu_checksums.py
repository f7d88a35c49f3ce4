"""CRC32 / Adler32 on the GPU through the C-ABI, against the oracle and the
reference-generated vectors."""
import pytest

from golden_util import load, make_input

pytestmark = pytest.mark.gpu

CK = load("checksums.json")


@pytest.fixture(scope="module")
def zt():
    import ztamd

    assert ztamd.device_count() > 0, "no GPU visible"
    return ztamd


@pytest.mark.parametrize("rec", [r for r in CK["records"] if r["input"].get("n", 0) < (1 << 24)],
                         ids=lambda r: str(r["input"])[:40])
def test_golden(zt, oracle, rec):
    d = make_input(rec["input"], oracle)
    assert zt.crc32(d) == rec["crc32"]
    assert zt.adler32(d) == rec["adler32"]
    c, a = zt.checksums(d)
    assert (c, a) == (rec["crc32"], rec["adler32"])
    if "crc32_chain" in rec:
        cut = len(d) >> 1
        assert zt.crc32(d[cut:], zt.crc32(d[:cut])) == rec["crc32_chain"]
        assert zt.adler32(d[cut:], zt.adler32(d[:cut])) == rec["adler32_chain"]


def test_one_gib_pin(zt, oracle):
    # config C1: 1 GiB xorshift32 seed 11 (SURVEY.md 8(d) pins)
    d = oracle.gen("xorshift32", 11, 1 << 30)
    assert zt.checksums(d) == (0x8EFD43CD, 0xC40E5752)


@pytest.mark.parametrize("n", [1, 7, 15, 16, 17, 1023, 1024, 1025, 262143, 262144, 262145, 3 * 262144 + 77,
                               (1 << 22) + 5])
@pytest.mark.parametrize("off", [0, 1, 13])
def test_ragged_and_unaligned(zt, oracle, n, off):
    d = oracle.gen("wordsalad", n + off, n + off)
    assert zt.checksums(d[off:]) == (oracle.crc32(d[off:]), oracle.adler32(d[off:]))


def test_init_values(zt, oracle):
    d = oracle.gen("structured", 3, 100000)
    for crc, adler in [(0, 1), (0xFFFFFFFF, 0xFFFFFFFF), (0x12345678, 0x0001FFF0), (7, 65521)]:
        assert zt.crc32(d, crc) == oracle.crc32(d, crc)
        assert zt.adler32(d, adler) == oracle.adler32(d, adler)
    # zero length returns the inputs untouched (no % 65521), like the reference
    assert zt.adler32(b"", 0xFFFFFFFF) == 0xFFFFFFFF
    assert zt.crc32(b"", 0xDEADBEEF) == 0xDEADBEEF


def test_device_resident(zt, oracle):
    import torch

    d = oracle.gen("xorshift32", 5, (1 << 24) + 3)
    t = torch.frombuffer(bytearray(d), dtype=torch.uint8).cuda()
    for off in (0, 1, 5):
        assert zt.dev_checksums(t.data_ptr() + off, len(d) - off) == (oracle.crc32(d[off:]), oracle.adler32(d[off:]))
