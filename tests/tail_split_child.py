"""Child process of tests/test_gpu_deflate.py::test_tail_split_streams_identical:
deflates the device-generated 48 MiB mixed corpus at level 6 under the
environment it was started with (ZT_DF_TAILK is read once per process) and
prints the stream's SHA-256 as JSON.  Test infrastructure only."""
import hashlib
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "zlib.ts_amd", "py"))
import torch  # noqa: E402
import ztamd as zt  # noqa: E402

n = 48 << 20
d_in = torch.empty(n, dtype=torch.uint8, device="cuda")
d_c = torch.empty(zt.deflate_bound(n), dtype=torch.uint8, device="cuda")
zt.synth_dev("mixed", 7, d_in.data_ptr(), n)
dp = zt.DeflatePlan(n, level=6)
clen = dp.run(d_in.data_ptr(), n, d_c.data_ptr())
dp.close()
torch.cuda.synchronize()
s = d_c[:clen].cpu().numpy().tobytes()
print(json.dumps({"len": clen, "sha256": hashlib.sha256(s).hexdigest()}), flush=True)
