"""Config C2 at its own workload: RawInflate of 4,096
distinct reference-deflated 64 KiB blocks in one zt_inflate_raw_batch call
(replaces src/RawInflate.ts:127-140,466-516 per stream).

* default mode: every output equals its input block and `.ip` equals the
  stream length (the reference's RawInflate ip: the byte after the last used
  bit, restated by the oracle);
* ref_strict mode: status, output, `.ip` and error text equal the
  reference's (oracle) for every stream, including the streams its
  over-strict EOF check rejects (src/RawInflate.ts:187)."""
import pytest

import c2_corpus

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def corpus(oracle):
    return c2_corpus.build(oracle)


@pytest.fixture(scope="module")
def zt():
    import ztamd

    assert ztamd.device_count() > 0, "no GPU visible"
    return ztamd


def test_c2_corpus_shape(corpus):
    assert len(corpus) == c2_corpus.COUNT
    assert len({s for _, s, _ in corpus}) == c2_corpus.COUNT  # distinct streams
    assert all(len(raw) == c2_corpus.BLOCK for raw, _, _ in corpus)


def test_c2_batch_default(zt, corpus):
    res = zt.inflate_raw_batch([s for _, s, _ in corpus])
    bad = []
    for i, ((raw, s, ref), (st, out, ip)) in enumerate(zip(corpus, res)):
        if st != 0 or out != raw or ip != len(s):
            bad.append((i, st, len(out), ip, len(s)))
        elif ref[0] == "ok":
            assert ref[1] and ref[2] == ip, i  # the reference decodes it to the same bytes and ip
    assert not bad, bad[:10]


def test_c2_batch_ref_strict(zt, corpus):
    import ztamd

    res = zt.inflate_raw_batch([s for _, s, _ in corpus], ref_strict=True)
    n_err = 0
    for i, ((raw, s, ref), (st, out, ip)) in enumerate(zip(corpus, res)):
        if ref[0] == "ok":
            assert st == 0 and out == raw and ip == ref[2], i
        else:
            n_err += 1
            assert st != 0, i
            with pytest.raises(ztamd.ZtError) as ei:
                zt.inflate_raw(s, ref_strict=True)
            assert ei.value.msg == ref[1], i
    print(f"C2: {n_err} of {len(corpus)} streams rejected by the reference's strict EOF check")
