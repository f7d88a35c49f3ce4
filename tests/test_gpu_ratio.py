"""Ratio gate of config C3: on each of the 16 fixed 4 MiB
windows (four per generator: wordsalad, xorshift32, structured, Python
stdlib source text) this build's RawDeflate at level 6 -- the bench level --
writes at most 1.02x the bytes of the reference's RawDeflate run on the
whole window with default options (src/RawDeflate.ts:87-114, src/LZ77.ts:
157-283; restated byte-exactly by the oracle).  Every stream is also
decoded by the reference's RawInflate restatement."""
import pytest

from ratio_corpus import reference_sizes, windows

pytestmark = pytest.mark.gpu

GATE = 1.02


@pytest.fixture(scope="module")
def gate_rows(oracle):
    import ztamd

    assert ztamd.device_count() > 0, "no GPU visible"
    wins = windows(oracle)
    refs = reference_sizes(oracle, wins)
    rows = []
    for (gen, label, data), ref in zip(wins, refs):
        s = ztamd.deflate_raw(data, level=6)
        out, _ = oracle.raw_inflate(s)
        assert out == data, label
        rows.append((gen, label, len(s), ref))
    for gen, label, ours, ref in rows:
        print(f"{label:24s} ours {ours:9d} ref {ref:9d} ratio {ours / ref:.4f}")
    return rows


def test_every_window_within_gate(gate_rows):
    bad = [(label, round(o / r, 4)) for _, label, o, r in gate_rows if o / r > GATE]
    assert not bad, bad


def test_per_generator_ratio(gate_rows):
    for gen in ["wordsalad", "xorshift32", "structured", "source"]:
        o = sum(x[2] for x in gate_rows if x[0] == gen)
        r = sum(x[3] for x in gate_rows if x[0] == gen)
        print(gen, round(o / r, 4))
        assert o / r <= GATE, gen


def test_adaptive_depth_engages_within_gate(oracle, gate_rows):
    """Level 6 chooses each block's search depth from its first 4 KiB
    (deflate.hip DeflateParams::adapt_depth): on the source-text and
    structured windows some blocks walk fewer hops than max_chain -- the
    streams differ from the fixed-depth ones (ZT_DF_ADAPT=0,0) -- and every
    window, adaptive or not, stays within the gate.  Streams decode through
    the reference's RawInflate restatement."""
    import os

    import ztamd

    wins = windows(oracle)
    gated = {label: (ours, ref) for _, label, ours, ref in gate_rows}
    differ = 0
    os.environ["ZT_DF_ADAPT"] = "0,0"
    try:
        for gen, label, data in wins:
            if gen not in ("source", "structured"):
                continue
            fixed = ztamd.deflate_raw(data, level=6)
            ours, ref = gated[label]
            assert len(fixed) / ref <= GATE and ours / ref <= GATE, label
            differ += len(fixed) != ours
    finally:
        del os.environ["ZT_DF_ADAPT"]
    assert differ > 0, "no block took the shallower depth"
