"""Config C4's workload: 10 000 seeded files, sizes
log-uniform 1 KiB - 1 MiB (mean ~148 KiB, ~1.41 GiB), half text (wordsalad
and slices of the Python standard-library sources, /usr/lib/python3.10, as
tests/ratio_corpus.py) and half binary (xorshift32 random and structured
small-delta int32).  Shared by tests/test_gpu_c4.py, its alias-device child
and tools/c4_batch.py, so every one of them compresses the same batch.
Test infrastructure: the generators are the oracle's (zo_gen)."""
import hashlib
import math
import random

from ratio_corpus import source_text

FILES = 10000


def c4_files(oracle, count=FILES, seed=1):
    rng = random.Random(seed)
    src = source_text()
    files = []
    for i in range(count):
        n = int(math.exp(rng.uniform(math.log(1 << 10), math.log(1 << 20))))
        if i % 2 == 0:  # text
            if i % 4 == 0:
                files.append(oracle.gen("wordsalad", seed * 100003 + i, n))
            else:
                off = rng.randrange(0, len(src) - n)
                files.append(src[off:off + n])
        else:  # binary
            files.append(oracle.gen("xorshift32" if i % 4 == 1 else "structured", seed * 100003 + i, n))
    return files


def members_digest(members):
    """sha256 over every member's length and bytes, in order."""
    h = hashlib.sha256()
    for m in members:
        h.update(len(m).to_bytes(8, "little"))
        h.update(m)
    return h.hexdigest()
