"""Config C2 of SURVEY.md 8(d), at its own workload: 4,096 distinct 64 KiB
blocks -- block i is xorshift32(100 + i) for even i and wordsalad(100 + i)
for odd i -- each deflated by the reference's RawDeflate (default options:
one dynamic block per input, src/RawDeflate.ts:87-114), restated byte-exactly
by the oracle (pinned by tests/test_oracle_golden.py).  The oracle also
decodes every stream with the reference's RawInflate (src/RawInflate.ts:
127-140, 466-516): its output, `.ip` and thrown error are what the GPU batch
must reproduce.  Shared by tests/test_gpu_c2.py and tools/c2_bench.py.

Test infrastructure only: the product path never imports this module.
"""
from concurrent.futures import ThreadPoolExecutor

COUNT = 4096
BLOCK = 65536
SEED0 = 100


def kind(i):
    return "xorshift32" if i % 2 == 0 else "wordsalad"


def _one(oracle, i):
    from zt_oracle import OracleError

    raw = oracle.gen(kind(i), SEED0 + i, BLOCK)
    s, _ = oracle.raw_deflate(raw)
    try:
        out, ip = oracle.raw_inflate(s)
        ref = ("ok", out == raw, ip)
    except OracleError as e:
        # the reference's over-strict EOF check (src/RawInflate.ts:187) rejects
        # some valid streams; its message is the expected strict-mode error
        ref = ("error", e.msg, None)
    return raw, s, ref


def build(oracle, count=COUNT, threads=16):
    """[(raw, stream, reference_result)] for blocks 0..count-1.  The oracle
    runs in threads (ctypes releases the GIL): ~0.07 s per block on one core."""
    with ThreadPoolExecutor(threads) as ex:
        return list(ex.map(lambda i: _one(oracle, i), range(count)))
