"""Config C4 host-side stage rates: zt_gzip_compress_batch
of the 10 000-file corpus (tests/c4_corpus.py) with the library's host-only
stage timers on (ZT_BATCH_STAGES=1: per device share, the wall time of
packing the buffers into pinned staging and of framing the members, on the
threads that do it), once on one device and once split over 8 logical
devices (ZT_ALIAS_DEVICES=8, zt_set_devices(0xFF): eight device contexts,
eight host threads, all running on the one physical GPU).  The host work of
an 8-GPU node keeps up when every device's pack + frame rate is at least
the one-GPU end-to-end C4 rate: the stages of different devices run on
different host threads.
   usage: python tools/c4_host_stages.py [files] [out.json]"""
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))

CHILD = r"""
import ctypes, json, os, sys, time
sys.path.insert(0, os.path.join(%(root)r, "tests")); sys.path.insert(0, os.path.join(%(root)r, "zlib.ts_amd", "py"))
import zt_oracle, ztamd
from c4_corpus import c4_files
files = c4_files(zt_oracle.Oracle(), %(count)d, 1)
k = len(files)
if %(mask)d: ztamd.set_devices(%(mask)d)
ptrs = (ctypes.c_void_p * k)(*[ctypes.cast(ctypes.c_char_p(x), ctypes.c_void_p).value for x in files])
lens = (ctypes.c_size_t * k)(*[len(x) for x in files])
opts = ztamd.GzipOpts(); opts.deflate = ztamd.DeflateOpts(2, 0, 6)
for rep in range(3):
    outs = (ctypes.POINTER(ctypes.c_uint8) * k)(); olens = (ctypes.c_size_t * k)(); st = (ctypes.c_int * k)()
    sys.stderr.write(json.dumps({"rep": rep}) + "\n"); sys.stderr.flush()
    t0 = time.perf_counter()
    ztamd._check(ztamd.lib.zt_gzip_compress_batch(ptrs, lens, k, ctypes.byref(opts), outs, olens, st))
    dt = time.perf_counter() - t0
    sys.stderr.write(json.dumps({"call_s": dt, "bytes": sum(len(f) for f in files)}) + "\n"); sys.stderr.flush()
    for i in range(k): ztamd.lib.zt_free(outs[i])
"""


def run(count, alias):
    env = dict(os.environ, ZT_BATCH_STAGES="1")
    if alias:
        env["ZT_ALIAS_DEVICES"] = str(alias)
    code = CHILD % {"root": os.path.join(HERE, ".."), "count": count, "mask": (1 << alias) - 1 if alias else 0}
    p = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=600)
    if p.returncode:
        raise SystemExit(p.stderr[-3000:])
    reps, cur = [], None
    for line in p.stderr.splitlines():
        if not line.startswith("{"):
            continue
        d = json.loads(line)
        if "rep" in d:
            cur = {"shares": []}
            reps.append(cur)
        elif "zt_batch_stages" in d:
            cur["shares"].append(d)
        elif "call_s" in d:
            cur.update(d)
    best = min(reps[1:] or reps, key=lambda r: r["call_s"])  # (rep 0 pays the allocations)
    gib = best["bytes"] / 2**30
    shares = best["shares"]
    for s in shares:
        s["pack_GiBps"] = round(s["in_bytes"] / 2**30 / (s["pack_ms"] / 1e3), 1) if s["pack_ms"] else None
        s["frame_GiBps"] = round(s["in_bytes"] / 2**30 / (s["frame_ms"] / 1e3), 1) if s["frame_ms"] else None
        s["host_GiBps"] = round(s["in_bytes"] / 2**30 / ((s["pack_ms"] + s["frame_ms"]) / 1e3), 1)
    return {"devices": alias or 1, "call_s": round(best["call_s"], 4), "GiBps": round(gib / best["call_s"], 2),
            "shares": shares}


def main():
    count = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
    res = {"files": count, "one": run(count, 0), "alias8": run(count, 8)}
    one = res["one"]["GiBps"]
    slow = min(s["host_GiBps"] for s in res["alias8"]["shares"])
    res["one_gpu_c4_GiBps"] = one
    res["slowest_device_host_GiBps"] = slow
    # per device, the host stages must beat that device's share of an
    # 8-GPU node's rate: 8 devices x one = the node, 1/8 of the data each
    res["host_keeps_up_with_8x"] = slow >= one
    print(json.dumps(res, indent=1))
    if len(sys.argv) > 2:
        with open(sys.argv[2], "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
