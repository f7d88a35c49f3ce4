#!/usr/bin/env python3
"""bench.py -- the headline metric of BASELINE.json on MI355X:

    "GiB/s RawDeflate L6 + RawInflate on 1 GiB buffer; ratio vs ref"

One step = RawDeflate (level 6) of a 1 GiB device-resident synthetic buffer
followed by RawInflate of the resulting stream back into HBM, both through
libzt's device entry points (zt_deflate_dev / zt_inflate_dev, include/zt.h).
The corpus is SURVEY.md 8(d)'s mixed generator set (wordsalad, xorshift32,
structured int32 deltas, cycling per 4 MiB window), generated on the device.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--size BYTES] [--level L]

For N > 1 the driver launches one process per GPU (torch.distributed.run);
every rank round-trips its own 1 GiB buffer (weak scaling, no collective on
the data path); the timed region is bracketed by barrier + synchronize and
the maximum over ranks is reported.  value = total bytes round-tripped by all
ranks / max elapsed.

Extra fields: `roofline` for the dominant kernel (deflate's match_kernel,
the LZ77 match finder; algorithmic bytes = N input bytes per launch, SURVEY.md
8(d), timed with HIP events on its launch stream), `cpu_baseline` (the oracle -- the
C restatement of the reference's RawDeflate + RawInflate -- on a bounded
sample, rank 0, N = 1 only), and the per-generator compression ratio of this
build against the reference on that sample.
"""
import argparse
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "zlib.ts_amd", "py"))

import torch  # noqa: E402

from zt_shard import max_over_ranks  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E, /opt/skills/guides/MI355X_MICROARCH.md
WINDOW = 4 << 20
KINDS = ["wordsalad", "xorshift32", "structured"]  # mixed corpus order per 4 MiB window


def cpu_baseline(d_in, level, zt):
    """Oracle (C restatement of src/RawDeflate.ts + src/RawInflate.ts, 1 core)
    on the first three 4 MiB windows of the bench corpus; also the ratio of
    this build's deflate to the reference's bytes per generator."""
    sys.path.insert(0, os.path.join(HERE, "tests"))
    import zt_oracle

    o = zt_oracle.Oracle()
    t_total = 0.0
    nbytes = 0
    ratios = {}
    for w, kind in enumerate(KINDS):
        chunk = bytes(d_in[w * WINDOW:(w + 1) * WINDOW].cpu().numpy())
        t0 = time.perf_counter()
        ref, _ = o.raw_deflate(chunk)
        back, _ = o.raw_inflate(ref)
        t_total += time.perf_counter() - t0
        assert back == chunk
        nbytes += len(chunk)
        ours = zt.deflate_raw(chunk, level=level)
        ratios[kind] = round(len(ours) / len(ref), 4)
    return {
        "value": round(nbytes / t_total / 2**30, 5),
        "unit": "GiB/s",
        "cores": 1,
        "kind": "port",
        "sample": "RawDeflate (reference defaults) + RawInflate of the first 3 x 4 MiB windows of the corpus "
                  "(wordsalad, xorshift32, structured), oracle/liboracle.so, single thread",
    }, ratios


def pmc_traffic(kernel, n):
    """HBM bytes per launch of `kernel` measured by rocprofv3 PMC passes
    (FETCH_SIZE x2 + WRITE_SIZE, tools/pmc_traffic.py) on this workload, or
    None when no measurement for this size is committed."""
    path = os.path.join(HERE, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            k = json.load(f)["kernels"][kernel]
    except (OSError, KeyError, ValueError):
        return None
    if n != 1 << 30:
        return None
    return int(k["traffic_bytes"])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--size", type=int, default=1 << 30)
    ap.add_argument("--level", type=int, default=6)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    import ztamd as zt

    zt.set_device(local)
    dist = None
    if world > 1:
        import torch.distributed as dist

        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    n = args.size
    d_in = torch.empty(n, dtype=torch.uint8, device="cuda")
    zt.synth_dev("mixed", 11 + 7919 * rank, d_in.data_ptr(), n)
    bound = zt.deflate_bound(n)
    d_c = torch.empty(bound, dtype=torch.uint8, device="cuda")
    d_out = torch.empty(n + 4096, dtype=torch.uint8, device="cuda")
    dplan = zt.DeflatePlan(n, level=args.level)
    iplan = zt.InflatePlan(bound, n)
    torch.cuda.synchronize()

    def step():
        clen = dplan.run(d_in.data_ptr(), n, d_c.data_ptr())
        olen, _ = iplan.run(d_c.data_ptr(), clen, d_out.data_ptr(), d_out.numel())
        return clen, olen

    # correctness of the measured path (untimed): the round trip is exact
    clen, olen = step()
    torch.cuda.synchronize()
    if olen != n or not torch.equal(d_out[:n], d_in):
        raise SystemExit("bench: round trip mismatch")
    for _ in range(args.warmup):
        step()

    def barrier():
        if dist is not None:
            dist.barrier()

    barrier()
    torch.cuda.synchronize()
    zt.timing_enable(True)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        clen, olen = step()
    torch.cuda.synchronize()
    barrier()
    elapsed = time.perf_counter() - t0
    kt = zt.timing_read()
    zt.timing_enable(False)
    elapsed = max_over_ranks(elapsed, dist, device="cuda")

    value = world * n * args.steps / elapsed / 2**30
    ms_step = elapsed / args.steps * 1e3
    def_ms = kt["deflate_ms"] / max(1, kt["deflate_launches"])  # match_kernel (dominant deflate kernel)
    pipe_ms = kt["deflate_pipeline_ms"] / max(1, kt["deflate_pipelines"])
    inf_ms = kt["inflate_ms"] / max(1, kt["inflate_launches"])
    tok_ms = kt["inflate_tok_ms"] / max(1, kt["inflate_toks"])
    achieved = n / (def_ms * 1e-3) / 1e9 if def_ms > 0 else 0.0
    line = {
        "metric": "GiB/s RawDeflate L6 + RawInflate on 1 GiB buffer; ratio vs ref",
        "value": round(value, 4),
        "unit": "GiB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_step, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (device-generated mixed corpus: wordsalad / xorshift32 / structured per 4 MiB window)",
        "config": {"workload": f"RawDeflate level {args.level} + RawInflate round trip of a {n / 2**30:g} GiB "
                               "device-resident buffer per GPU", "bytes_per_gpu": n, "level": args.level,
                   "parallelism": f"batch split x{world} (no collective)"},
        "ratio": round(clen / n, 5),
        "match_kernel_ms": round(def_ms, 3),
        "deflate_pipeline_ms": round(pipe_ms, 3),
        "inflate_kernel_ms": round(inf_ms, 3),
        "inflate_tokenize_ms": round(tok_ms, 3),
        "deflate_GiBps": round(n / (pipe_ms * 1e-3) / 2**30, 3) if pipe_ms else None,
        "inflate_GiBps": round(n / (inf_ms * 1e-3) / 2**30, 3) if inf_ms else None,
        "roofline": {"bound": "hbm", "kernel": "match_kernel", "achieved": round(achieved, 3),
                     "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 6),
                     "traffic": pmc_traffic("match_kernel", n)},
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline and n >= 3 * WINDOW:
        cb, ratios = cpu_baseline(d_in, args.level, zt)
        line["cpu_baseline"] = cb
        line["ratio_vs_ref"] = ratios
    if rank == 0:
        print(json.dumps(line), flush=True)
    dplan.close()
    iplan.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
