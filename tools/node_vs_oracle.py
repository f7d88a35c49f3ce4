"""Speed of the C restatement (oracle/, bench.py's cpu_baseline, kind "port")
relative to the reference itself in Node (tools/node_vs_oracle.mjs), on the
same sample: three 4 MiB windows (wordsalad, xorshift32, structured), one
host core each.  Writes profiles/node_vs_oracle.json.  Needs /root/reference
(this container only)."""
import json
import os
import subprocess
import sys
import tempfile
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "tests"))
import zt_oracle  # noqa: E402

o = zt_oracle.Oracle()
wins = [o.gen(k, 1, 4 << 20) for k in ("wordsalad", "xorshift32", "structured")]
d = tempfile.mkdtemp()
files = []
for i, w in enumerate(wins):
    files.append(os.path.join(d, f"w{i}.bin"))
    with open(files[-1], "wb") as f:
        f.write(w)
node = json.loads(subprocess.check_output(["node", os.path.join(HERE, "node_vs_oracle.mjs")] + files).decode().splitlines()[-1])
tdef = tinf = 0.0
comp = 0
for w in wins:
    t0 = time.perf_counter()
    s, _ = o.raw_deflate(w)
    t1 = time.perf_counter()
    back, _ = o.raw_inflate(s)
    t2 = time.perf_counter()
    assert back == w
    comp += len(s)
    tdef += t1 - t0
    tinf += t2 - t1
n = sum(len(w) for w in wins)
res = {
    "sample": "3 x 4 MiB windows (wordsalad, xorshift32, structured), one core",
    "node": node["node"],
    "reference_node": {"deflate_MiBps": round(n / node["deflate_s"] / 2**20, 2),
                       "inflate_MiBps": round(n / node["inflate_s"] / 2**20, 2),
                       "roundtrip_MiBps": round(n / (node["deflate_s"] + node["inflate_s"]) / 2**20, 2),
                       "compressed": node["compressed"]},
    "oracle_c": {"deflate_MiBps": round(n / tdef / 2**20, 2), "inflate_MiBps": round(n / tinf / 2**20, 2),
                 "roundtrip_MiBps": round(n / (tdef + tinf) / 2**20, 2), "compressed": comp},
}
res["oracle_over_node_roundtrip"] = round(res["oracle_c"]["roundtrip_MiBps"] / res["reference_node"]["roundtrip_MiBps"], 3)
out = os.path.join(HERE, "..", "profiles", "node_vs_oracle.json")
with open(out, "w") as f:
    json.dump(res, f, indent=1)
print(json.dumps(res))
