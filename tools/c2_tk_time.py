# Tokenizer phase cycles of the C2 batch per generator (libzt built with
# -DZT_TK_TIME, ZT_LIB=...): COUNT reference-deflated 64 KiB streams of one
# kind (tests/c2_corpus.py's seeds), one zt_inflate_raw_batch call, cycles per
# round of 64 x 480 bits: staging / pass 1 / repairs (phase maps inside) / pass 2.
#   usage: python tools/c2_tk_time.py [count]
import ctypes, os, sys, time
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "zlib.ts_amd", "py"))
sys.path.insert(0, os.path.join(HERE, "..", "tests"))
import c2_corpus  # noqa: E402
import ztamd as zt  # noqa: E402
import zt_oracle  # noqa: E402
count = int(sys.argv[1]) if len(sys.argv) > 1 else 512
o = zt_oracle.Oracle()
buf = (ctypes.c_ulonglong * 8)()
for par in (0, 1):
    idx = [2 * i + par for i in range(count)]
    streams = []
    raws = []
    for i in idx:
        raw, s, _ = c2_corpus._one(o, i)
        raws.append(raw)
        streams.append(s)
    res = zt.inflate_raw_batch(streams)
    assert all(st == 0 and ob == r for (st, ob, ip), r in zip(res, raws))
    zt.lib.zt_debug_tk_time(buf)
    t0 = time.perf_counter()
    zt.inflate_raw_batch(streams)
    dt = time.perf_counter() - t0
    zt.lib.zt_debug_tk_time(buf)
    r = max(1, buf[4])
    print(f"{c2_corpus.kind(idx[0]):10s} {count} streams, call {dt*1e3:.1f} ms: {buf[4]} rounds, "
          f"{buf[5] / r:.2f} repair iterations per round; cycles per round: "
          f"stage {buf[0] / r:.0f} (store wait {buf[7] / r:.0f})  pass1 {buf[1] / r:.0f}  repairs {buf[2] / r:.0f} (maps {buf[6] / r:.0f})  "
          f"pass2 {buf[3] / r:.0f}", flush=True)
