"""Timing of the general parallel inflate (csrc/inflate_gen.hip) on streams
without sync points: a reference-style single-block stream (the oracle's
restatement of src/RawDeflate.ts, one dynamic block) and zlib level-6 raw
streams of the mixed corpus.  Device-resident (zt_inflate_dev through the
inflate plan, wall time around the call = everything incl. the host chain
passes) and host API (zt_inflate_raw, PCIe included; cold first call and
the best warm call).
   usage: python tools/inflate_general_time.py [MiB] [out.json]"""
import json
import os
import sys
import time
import zlib

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "tests"))
sys.path.insert(0, os.path.join(HERE, "..", "zlib.ts_amd", "py"))
import torch  # noqa: E402

import zt_oracle  # noqa: E402
import ztamd  # noqa: E402


def mixed(o, n, seed):
    kinds = ["wordsalad", "xorshift32", "structured"]
    parts, i = [], 0
    while sum(len(p) for p in parts) < n:
        parts.append(o.gen(kinds[(seed + i) % 3], seed * 101 + i, 1 << 20))
        i += 1
    return b"".join(parts)[:n]


def time_dev(s, d, reps=5):
    di = torch.frombuffer(bytearray(s), dtype=torch.uint8).cuda()
    do = torch.empty(len(d) + 4096, dtype=torch.uint8, device="cuda")
    p = ztamd.InflatePlan(len(s), len(d))
    p.run(di.data_ptr(), len(s), do.data_ptr(), do.numel())
    torch.cuda.synchronize()
    assert bytes(do[:len(d)].cpu().numpy()) == d
    ztamd.timing_enable(True)
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        olen, ip = p.run(di.data_ptr(), len(s), do.data_ptr(), do.numel())
        ts.append(time.perf_counter() - t0)
        assert olen == len(d) and ip == len(s)
    t = ztamd.timing_read()
    ztamd.timing_enable(False)
    best = min(ts)
    return {"wall_ms": round(best * 1e3, 3), "GiBps": round(len(d) / best / 2**30, 3),
            "event_ms": round(t["inflate_ms"] / max(t["inflate_launches"], 1), 3),
            "paths": t["inflate_paths"], "passes_per_call": t["general_passes"] / max(t["inflate_paths"][1], 1)}


def time_api(s, data, reps=3):
    """zt_inflate_raw of the host stream into a library output (PCIe
    included), C-ABI through ctypes: the first (cold: scratch, staging and
    output allocations) call, then the best of `reps` warm calls (outputs
    handed back with zt_free, as a looping caller does)."""
    import ctypes

    import numpy as np

    src = np.frombuffer(s, dtype=np.uint8)
    iopts = ztamd.InflateOpts(1, 0x8000, 0)
    ts = []
    for rep in range(reps + 1):
        back = ctypes.POINTER(ctypes.c_uint8)()
        blen, ip = ctypes.c_size_t(), ctypes.c_size_t()
        t0 = time.perf_counter()
        ztamd._check(ztamd.lib.zt_inflate_raw(src.ctypes.data_as(ctypes.c_void_p), len(s), 0, ctypes.byref(iopts),
                                              ctypes.byref(back), ctypes.byref(blen), ctypes.byref(ip)))
        ts.append(time.perf_counter() - t0)
        assert blen.value == len(data) and ip.value == len(s)
        if rep == 0:
            assert ctypes.string_at(back, blen.value) == data
        ztamd.lib.zt_free(back)
    return {"host_api_GiBps": round(len(data) / min(ts[1:]) / 2**30, 3),
            "host_api_cold_GiBps": round(len(data) / ts[0] / 2**30, 3),
            "host_api_ms": [round(t * 1e3, 2) for t in ts]}


def main():
    mib = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    out_json = sys.argv[2] if len(sys.argv) > 2 else None
    o = zt_oracle.Oracle()
    data = mixed(o, mib << 20, 5)
    res = {"bytes": len(data)}
    t0 = time.perf_counter()
    ref, _ = o.raw_deflate(data)
    res["oracle_deflate_s"] = round(time.perf_counter() - t0, 2)
    print("oracle deflate done", res["oracle_deflate_s"], flush=True)
    t0 = time.perf_counter()
    back, ip = o.raw_inflate(ref)
    dt = time.perf_counter() - t0
    assert back == data and ip == len(ref)
    res["cpu_oracle_inflate_MiBps"] = round(len(data) / dt / 2**20, 1)
    print("oracle inflate", res["cpu_oracle_inflate_MiBps"], "MiB/s", flush=True)
    streams = {"reference_single_block": ref}
    c = zlib.compressobj(6, zlib.DEFLATED, -15)
    streams["zlib_l6"] = c.compress(data) + c.flush()
    c = zlib.compressobj(1, zlib.DEFLATED, -15)
    streams["zlib_l1"] = c.compress(data) + c.flush()
    for name, s in streams.items():
        r = {"stream_bytes": len(s)}
        print(name, len(s), flush=True)
        r["device"] = time_dev(s, data)
        print(name, "device", r["device"], flush=True)
        r.update(time_api(s, data))
        print(name, "host api", r["host_api_GiBps"], "(cold", r["host_api_cold_GiBps"], ")", flush=True)
        t0 = time.perf_counter()
        zlib.decompress(s, -15)
        r["cpu_zlib_MiBps"] = round(len(data) / (time.perf_counter() - t0) / 2**20, 1)
        res[name] = r
        print(name, json.dumps(r), flush=True)
    if out_json:
        with open(out_json, "w") as f:
            json.dump(res, f, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
