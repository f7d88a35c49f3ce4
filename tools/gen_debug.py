"""Debug: the general inflate of a reference-style single-block stream vs its
input -- first mismatching byte, output length.   usage: python tools/gen_debug.py MiB [seed]"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "tests"))
sys.path.insert(0, os.path.join(HERE, "..", "zlib.ts_amd", "py"))
import torch  # noqa: E402

import zt_oracle  # noqa: E402
import ztamd  # noqa: E402
from inflate_general_time import mixed  # noqa: E402

mib = int(sys.argv[1]) if len(sys.argv) > 1 else 64
seed = int(sys.argv[2]) if len(sys.argv) > 2 else 5
o = zt_oracle.Oracle()
data = mixed(o, mib << 20, seed)
s, _ = o.raw_deflate(data)
print("stream", len(s), flush=True)
di = torch.frombuffer(bytearray(s), dtype=torch.uint8).cuda()
do = torch.zeros(len(data) + 4096, dtype=torch.uint8, device="cuda")
p = ztamd.InflatePlan(len(s), len(data))
olen, ip = p.run(di.data_ptr(), len(s), do.data_ptr(), do.numel())
torch.cuda.synchronize()
got = bytes(do[:len(data)].cpu().numpy())
print("olen", olen, "want", len(data), "ip", ip, len(s), flush=True)
if got != data:
    i = next(k for k in range(len(data)) if got[k] != data[k])
    bad = sum(1 for k in range(i, min(len(data), i + (1 << 20))) if got[k] != data[k])
    print("first mismatch at", i, "bad bytes in next MiB", bad, flush=True)
    print("got ", got[i - 8:i + 24].hex(), "\nwant", data[i - 8:i + 24].hex())
else:
    print("OK")
if len(sys.argv) > 3:
    from pyinflate_tokens import tokens_from
    pos = int(sys.argv[3])
    for p0, t in tokens_from(s, pos, int(sys.argv[4]) if len(sys.argv) > 4 else 60):
        print("PYTOK", p0, hex(t) if t >= 0 else "EOB")
