"""Secondary measurements for BASELINE.json configs other than the headline:
  C1  CRC32 + Adler32 over a 1 GiB device-resident buffer (fused kernel)
  C2  RawInflate batch: 4096 independent 64 KiB streams (host API, PCIe included,
      and the device decode time of the batch)
  C3  RawDeflate level 6 of one 8 GiB device-resident buffer (deflate only), ratio
  C4  GZip of 10,000 mixed text/binary files (1-64 KiB) through the host API
      zt_gzip_compress (PCIe included), members checked by GUnzip
Streams for C2 are SURVEY 8(d)'s 4096 distinct blocks (tests/c2_corpus.py:
even i xorshift32(100 + i), odd i wordsalad(100 + i), each deflated by the
oracle's byte-exact restatement of the reference RawDeflate)."""
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
# C2: SURVEY 8(d)'s workload -- 4096 distinct reference-deflated 64 KiB blocks
# (tests/c2_corpus.py; the device-side kernel times: tools/c2_bench.py under rocprofv3)
o = zt_oracle.Oracle()
import c2_corpus
corpus = c2_corpus.build(o)
streams = [s for _, s, _ in corpus]
out = zt.inflate_raw_batch(streams)
assert all(st == 0 and ob == raw for (raw, _, _), (st, ob, ip) in zip(corpus, out))
t0 = time.perf_counter()
for _ in range(3):
    zt.inflate_raw_batch(streams)
dt = (time.perf_counter() - t0) / 3
res["C2_batch_inflate_GiBps_host_api"] = round(4096 * 65536 / dt / 2**30, 3)
res["C2_input_MiB"] = round(sum(len(s) for s in streams) / 2**20, 1)
print(json.dumps(res), flush=True)
# C3
n = 8 << 30
d = torch.empty(n, dtype=torch.uint8, device="cuda")
zt.synth_dev("mixed", 17, d.data_ptr(), n)
dc = torch.empty(zt.deflate_bound(n), dtype=torch.uint8, device="cuda")
plan = zt.DeflatePlan(n)
torch.cuda.synchronize()
clen = plan.run(d.data_ptr(), n, dc.data_ptr())
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(2):
    clen = plan.run(d.data_ptr(), n, dc.data_ptr())
torch.cuda.synchronize()
dt = (time.perf_counter() - t0) / 2
res["C3_deflate_8GiB_GiBps"] = round(n / dt / 2**30, 2)
res["C3_ratio"] = round(clen / n, 5)
plan.close()
del d, dc
torch.cuda.empty_cache()
# C4
import random
rng = random.Random(4)
files = []
for i in range(10000):
    kind = ["wordsalad", "structured", "xorshift32"][i % 3]
    files.append(o.gen(kind, 9000 + i, rng.randint(1024, 65536)))
t0 = time.perf_counter()
members = [zt.gzip_compress(f, name=b"f%05d" % i, mtime=i)[0] for i, f in enumerate(files)]
dt = time.perf_counter() - t0
tot = sum(len(f) for f in files)
res["C4_gzip_files_per_s"] = round(len(files) / dt, 1)
res["C4_gzip_GiBps_host_api"] = round(tot / dt / 2**30, 3)
res["C4_input_MiB"] = round(tot / 2**20, 1)
res["C4_ratio"] = round(sum(len(m) for m in members) / tot, 4)
back, mems = zt.gunzip(b"".join(members[:200]))
assert back == b"".join(files[:200]) and len(mems) == 200
print(json.dumps(res), flush=True)
