"""The ratio-gate corpus of SURVEY.md 8(d): 16 fixed 4 MiB windows, four per
generator -- wordsalad, xorshift32, structured (small-delta LE int32) and
"source text" (Python 3.10 standard-library sources, /usr/lib/python3.10,
present in this image here and on the GPU box).  Shared by the GPU ratio
test and tools/ratio_gate.py.

The reference bytes of a window are the reference's RawDeflate run on the
whole window with default options (DYNAMIC, lazy 0), through its byte-exact
restatement in oracle/ (pinned by tests/test_oracle_golden.py).
"""
import glob
import os

WINDOW = 4 << 20
STDLIB = "/usr/lib/python3.10"
GENERATORS = ["wordsalad", "xorshift32", "structured", "source"]
SEEDS = [101, 102, 103, 104]


def source_text():
    """Top-level stdlib modules (SURVEY's definition: the first 4 MiB of the
    concatenated /usr/lib/python3.10/*.py), then the package modules, each
    group in sorted order."""
    top = sorted(glob.glob(os.path.join(STDLIB, "*.py")))
    sub = sorted(p for p in glob.glob(os.path.join(STDLIB, "*", "**", "*.py"), recursive=True)
                 if "-packages" not in p)
    out = bytearray()
    for p in top + sub:
        with open(p, "rb") as f:
            out += f.read()
    return bytes(out)


def windows(oracle):
    """[(generator, label, bytes)] -- the 16 windows, in a fixed order."""
    res = []
    for kind in ["wordsalad", "xorshift32", "structured"]:
        for s in SEEDS:
            res.append((kind, f"{kind}:{s}", oracle.gen(kind, s, WINDOW)))
    src = source_text()
    if len(src) < 2 * WINDOW:
        raise RuntimeError(f"{STDLIB} holds {len(src)} bytes of sources, the gate needs >= {2 * WINDOW}")
    # windows at 0 (the survey's "first 4 MiB"), then spread evenly over the rest (they overlap)
    step = (len(src) - WINDOW) // 3
    for k in range(4):
        off = k * step
        res.append(("source", f"source@{off}", src[off:off + WINDOW]))
    return res


def reference_sizes(oracle, wins, threads=16):
    """Reference RawDeflate output size of every window (the restatement runs
    in parallel threads: ctypes releases the GIL)."""
    from concurrent.futures import ThreadPoolExecutor

    def one(w):
        return len(oracle.raw_deflate(w[2])[0])

    with ThreadPoolExecutor(threads) as ex:
        return list(ex.map(one, wins))
