"""Config C2 measured at its own workload: zt_inflate_raw_batch
of the 4096 distinct reference-deflated 64 KiB blocks of tests/c2_corpus.py.

Prints one JSON line: the host-API rate (the C call alone: pinned packing,
H2D, the batch kernels, D2H and the output slab included; the Python
wrapper's time, with its byte copies, beside it) and, with ZT_BATCH_TIMING=1,
the stage split on stderr.  Run under `rocprofv3 --kernel-trace --stats` for
the device-side kernel times (sum of the batch kernels / CALLS = the device
time of one call; profiles/r03*_c2_*).
   usage: python tools/c2_bench.py [calls]
"""
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "zlib.ts_amd", "py"))
sys.path.insert(0, os.path.join(HERE, "..", "tests"))
import c2_corpus  # noqa: E402
import ztamd as zt  # noqa: E402
import zt_oracle  # noqa: E402

calls = int(sys.argv[1]) if len(sys.argv) > 1 else 5
t0 = time.perf_counter()
corpus = c2_corpus.build(zt_oracle.Oracle())
t_build = time.perf_counter() - t0
streams = [s for _, s, _ in corpus]
out = zt.inflate_raw_batch(streams)  # warm + check
ok = all(st == 0 and ob == raw and ip == len(s) for (raw, s, _), (st, ob, ip) in zip(corpus, out))
if not ok:
    raise SystemExit("c2_bench: mismatch")
ts = []
for _ in range(calls):
    t0 = time.perf_counter()
    zt.inflate_raw_batch(streams)
    ts.append(time.perf_counter() - t0)
# the C call alone: pointer arrays built once, outputs freed after the clock
# (the wrapper above also copies every input into a bytes object and every
# output into a new one)
import ctypes  # noqa: E402

k = len(streams)
bs = [bytes(x) for x in streams]
ptrs = (ctypes.c_void_p * k)(*[ctypes.cast(ctypes.c_char_p(x), ctypes.c_void_p).value for x in bs])
lens = (ctypes.c_size_t * k)(*[len(x) for x in bs])
opts = zt.InflateOpts(1, 0x8000, 0)
tc = []
for _ in range(calls + 1):
    outs = (ctypes.POINTER(ctypes.c_uint8) * k)()
    olens = (ctypes.c_size_t * k)()
    ips = (ctypes.c_size_t * k)()
    st = (ctypes.c_int * k)()
    t0 = time.perf_counter()
    rc = zt.lib.zt_inflate_raw_batch(ptrs, lens, k, ctypes.byref(opts), outs, olens, ips, st)
    tc.append(time.perf_counter() - t0)
    if rc != 0 or any(st[i] != 0 or olens[i] != c2_corpus.BLOCK or ips[i] != lens[i] for i in range(k)):
        raise SystemExit("c2_bench: C call failed")
    for i in range(k):
        zt.lib.zt_free(outs[i])
tc = sorted(tc[1:])
nbytes = c2_corpus.COUNT * c2_corpus.BLOCK
print(json.dumps({
    "config": "C2: zt_inflate_raw_batch of 4096 distinct reference-deflated 64 KiB blocks "
              "(even i xorshift32(100+i), odd i wordsalad(100+i))",
    "calls": calls,
    "input_MiB": round(sum(len(s) for s in streams) / 2**20, 2),
    "output_MiB": nbytes / 2**20,
    "host_api_ms_median": round(tc[len(tc) // 2] * 1e3, 2),
    "host_api_GiBps": round(nbytes / tc[len(tc) // 2] / 2**30, 3),
    "python_wrapper_ms_median": round(sorted(ts)[len(ts) // 2] * 1e3, 2),
    "corpus_build_s": round(t_build, 1),
}), flush=True)
