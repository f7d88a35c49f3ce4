"""Child process of tests/test_gpu_c4.py::test_c4_alias_devices: with
ZT_ALIAS_DEVICES set the library presents that many logical devices on the
one GPU (one context and host thread each); the C4 batch is compressed spread
over all of them by zt_set_devices (LPT split, batch_api.cpp run_batch) and
the members' digest is printed as JSON.  Test infrastructure only."""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(HERE, "..", "zlib.ts_amd", "py"))
import ztamd as zt  # noqa: E402
import zt_oracle  # noqa: E402
from c4_corpus import c4_files, members_digest  # noqa: E402

files = c4_files(zt_oracle.Oracle())
ndev = zt.device_count()
zt.set_devices((1 << ndev) - 1)
try:
    members = zt.gzip_compress_batch(files, mtime=0)
finally:
    zt.set_devices(0)
print(json.dumps({"logical_devices": ndev, "members": len(members), "digest": members_digest(members)}), flush=True)
