"""Device corpus generator (zt_synth_dev) equals the oracle's generators
piece by piece (64 KiB piece i = generator seeded with seed + i)."""
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("kind", ["xorshift32", "wordsalad", "structured", "mixed"])
def test_synth_matches_oracle(oracle, kind):
    import torch
    import ztamd

    n = (130 << 16) + 4321  # crosses a 4 MiB window (mixed) and ends mid-piece
    d = torch.zeros(n + 64, dtype=torch.uint8, device="cuda")
    ztamd.synth_dev(kind, 500, d.data_ptr(), n)
    got = bytes(d[:n].cpu().numpy())
    names = ["wordsalad", "xorshift32", "structured"]
    for i in range(0, (n + 65535) // 65536):
        k = names[(i >> 6) % 3] if kind == "mixed" else kind
        want = oracle.gen(k, 500 + i, min(65536, n - i * 65536))
        assert got[i * 65536:i * 65536 + len(want)] == want, (kind, i)
    assert bytes(d[n:].cpu().numpy()) == b"\0" * 64


def test_kernel_timing():
    import torch
    import ztamd

    n = 4 << 20
    d = torch.empty(n, dtype=torch.uint8, device="cuda")
    ztamd.synth_dev("mixed", 1, d.data_ptr(), n)
    c = torch.empty(ztamd.deflate_bound(n), dtype=torch.uint8, device="cuda")
    o = torch.empty(n, dtype=torch.uint8, device="cuda")
    dp, ip = ztamd.DeflatePlan(n), ztamd.InflatePlan(c.numel(), n)
    ztamd.timing_enable(True)
    clen = dp.run(d.data_ptr(), n, c.data_ptr())
    olen, _ = ip.run(c.data_ptr(), clen, o.data_ptr(), n)
    t = ztamd.timing_read()
    ztamd.timing_enable(False)
    assert olen == n and torch.equal(o, d)
    assert t["deflate_launches"] == 1 and t["deflate_ms"] > 0
    assert t["inflate_launches"] == 1 and t["inflate_ms"] > 0
