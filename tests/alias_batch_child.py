"""Child process of tests/test_gpu_batch.py::test_alias_devices_split: runs
with ZT_ALIAS_DEVICES set (the library then presents that many logical
devices on the one GPU, each with its own context), compresses one batch on
logical device 0 alone and again spread over every logical device by
zt_set_devices (LPT split, one host thread per device: batch_api.cpp
run_batch), and prints a JSON verdict.  Test infrastructure only."""
import json
import math
import os
import random
import sys
import zlib

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(HERE, "..", "zlib.ts_amd", "py"))
import ztamd as zt  # noqa: E402
import zt_oracle  # noqa: E402

o = zt_oracle.Oracle()
ndev = zt.device_count()
rng = random.Random(int(sys.argv[1]) if len(sys.argv) > 1 else 3)
kinds = ["wordsalad", "xorshift32", "structured"]
files = [b"", b"x", b"\0" * 32769]
while len(files) < 96:
    n = int(math.exp(rng.uniform(math.log(1 << 10), math.log(1 << 20))))
    files.append(o.gen(kinds[len(files) % 3], 4000 + len(files), n))
res = {"logical_devices": ndev}
single_gz = zt.gzip_compress_batch(files, mtime=7)
single_raw = zt.deflate_raw_batch(files)
single_crc = zt.crc32_batch(files)
zt.set_devices((1 << ndev) - 1)
try:
    split_gz = zt.gzip_compress_batch(files, mtime=7)
    split_raw = zt.deflate_raw_batch(files)
finally:
    zt.set_devices(0)
res["gzip_equal"] = split_gz == single_gz
res["raw_equal"] = split_raw == single_raw
ok = True
for f, m, s in zip(files, split_gz, split_raw):
    head = o.gzip_header(mtime=7)
    body, ip = o.raw_inflate(m, index=len(head))
    ok &= m[:len(head)] == head and body == f
    ok &= m[ip:ip + 4] == o.crc32(f).to_bytes(4, "little")
    ok &= zlib.decompress(s, -15) == f
res["oracle_ok"] = bool(ok)
res["crc_ok"] = single_crc == [o.crc32(f) for f in files]
print(json.dumps(res), flush=True)
