"""Secondary measurements for BASELINE.json configs other than the headline:
  C1  CRC32 + Adler32 over a 1 GiB device-resident buffer (fused kernel)
  C2  RawInflate batch: 4096 independent 64 KiB streams (host API, PCIe included,
      and the device decode time of the batch)
Streams for C2 are single-block raw DEFLATE of 64 KiB pieces produced by the
oracle's restatement of the reference RawDeflate (src/RawDeflate.ts: one
dynamic block per input), 64 distinct pieces replicated to 4096."""
import os, sys, time, json
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, '..', 'zlib.ts_amd', 'py')); sys.path.insert(0, os.path.join(HERE, '..', 'tests'))
import torch, ztamd as zt, zt_oracle

res = {}
# C1
n = 1 << 30
d = torch.empty(n, dtype=torch.uint8, device="cuda")
zt.synth_dev("mixed", 3, d.data_ptr(), n)
torch.cuda.synchronize()
crc, ad = zt.dev_checksums(d.data_ptr(), n)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(10):
    zt.dev_checksums(d.data_ptr(), n)
torch.cuda.synchronize()
dt = (time.perf_counter() - t0) / 10
res["C1_checksums_GiBps"] = round(n / dt / 2**30, 2)
res["C1_checksums_frac_hbm"] = round(n / dt / 8e12, 3)
del d
# C2
o = zt_oracle.Oracle()
pieces = []
for i in range(64):
    kind = ["wordsalad", "structured", "xorshift32"][i % 3]
    raw = o.gen(kind, 500 + i, 65536)
    s, _ = o.raw_deflate(raw)
    pieces.append((raw, s))
items = [pieces[i % 64] for i in range(4096)]
streams = [s for _, s in items]
out = zt.inflate_raw_batch(streams)
assert all(st == 0 and ob == raw for (raw, _), (st, ob, ip) in zip(items, out))
t0 = time.perf_counter()
for _ in range(3):
    zt.inflate_raw_batch(streams)
dt = (time.perf_counter() - t0) / 3
res["C2_batch_inflate_GiBps_host_api"] = round(4096 * 65536 / dt / 2**30, 3)
res["C2_input_MiB"] = round(sum(len(s) for s in streams) / 2**20, 1)
print(json.dumps(res), flush=True)
