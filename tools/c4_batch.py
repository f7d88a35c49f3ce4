"""Config C4: GZip end-to-end of a 10 000-file batch, sizes
log-uniform 1 KiB - 1 MiB, half text / half binary (tests/c4_corpus.py, the
batch tests/test_gpu_c4.py checks), through zt_gzip_compress_batch
(host buffers in, malloc'd members out: PCIe and host framing included) on
every visible GPU (zt_set_devices) -- and on one.  Members are verified with
zlib (an independent inflater) and a sample with the oracle's RawInflate.
   usage: python tools/c4_batch.py [files] [out.json]"""
import ctypes
import json
import os
import random
import sys
import time
import zlib

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "tests"))
sys.path.insert(0, os.path.join(HERE, "..", "zlib.ts_amd", "py"))
import zt_oracle  # noqa: E402
import ztamd  # noqa: E402
from c4_corpus import c4_files  # noqa: E402


def corpus(o, count, seed=1):
    return c4_files(o, count, seed)


def run(files, reps=3):
    k = len(files)
    ptrs = (ctypes.c_void_p * k)(*[ctypes.cast(ctypes.c_char_p(x), ctypes.c_void_p).value for x in files])
    lens = (ctypes.c_size_t * k)(*[len(x) for x in files])
    opts = ztamd.GzipOpts()
    opts.deflate = ztamd.DeflateOpts(2, 0, 6)
    best, members = None, None
    for _ in range(reps):
        outs = (ctypes.POINTER(ctypes.c_uint8) * k)()
        olens = (ctypes.c_size_t * k)()
        st = (ctypes.c_int * k)()
        t0 = time.perf_counter()
        rc = ztamd.lib.zt_gzip_compress_batch(ptrs, lens, k, ctypes.byref(opts), outs, olens, st)
        dt = time.perf_counter() - t0
        ztamd._check(rc)
        if members is None:
            members = [ctypes.string_at(outs[i], olens[i]) for i in range(k)]
        for i in range(k):
            ztamd.lib.zt_free(outs[i])
        best = dt if best is None else min(best, dt)
    return best, members


def main():
    count = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
    out_json = sys.argv[2] if len(sys.argv) > 2 else None
    o = zt_oracle.Oracle()
    t0 = time.perf_counter()
    files = corpus(o, count)
    total = sum(len(f) for f in files)
    print(f"corpus: {count} files, {total / 2**30:.3f} GiB ({time.perf_counter() - t0:.1f} s)", flush=True)
    ndev = ztamd.device_count()
    res = {"files": count, "bytes": total, "devices_visible": ndev}
    for nd in sorted({1, ndev}):
        ztamd.set_devices((1 << nd) - 1)
        ztamd.timing_enable(True)
        dt, members = run(files)
        t = ztamd.timing_read()
        ztamd.timing_enable(False)
        comp = sum(len(m) for m in members)
        r = {"seconds": round(dt, 4), "GiBps": round(total / dt / 2**30, 3), "files_per_s": round(count / dt, 1),
             "ratio": round(comp / total, 5),
             "deflate_pipeline_ms_per_call": round(t["deflate_pipeline_ms"] / max(t["deflate_pipelines"], 1), 3)}
        print(f"{nd} GPU(s):", json.dumps(r), flush=True)
        bad = 0
        for f, m in zip(files, members):
            if zlib.decompress(m, 31) != f:
                bad += 1
        rng = random.Random(3)
        for i in rng.sample(range(count), min(50, count)):
            body, ip = o.raw_inflate(members[i], index=10)
            if body != files[i] or members[i][ip:ip + 4] != o.crc32(files[i]).to_bytes(4, "little"):
                bad += 1
        r["verify_failures"] = bad
        res[f"gpus_{nd}"] = r
        print(f"{nd} GPU(s) verified, failures: {bad}", flush=True)
    ztamd.set_devices(0)
    # the r1 way for comparison: one zt_gzip_compress call per file (first 500)
    t0 = time.perf_counter()
    sub = files[:500]
    for f in sub:
        ztamd.gzip_compress(f)
    dt = time.perf_counter() - t0
    res["one_call_per_file_files_per_s"] = round(len(sub) / dt, 1)
    print(json.dumps(res), flush=True)
    if out_json:
        with open(out_json, "w") as fh:
            json.dump(res, fh, indent=1)


if __name__ == "__main__":
    main()
