# C4 per-call breakdown: GZip of 300 mixed files (1-64 KiB) through the host API
import os, sys, time, random
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, '..', 'zlib.ts_amd', 'py')); sys.path.insert(0, os.path.join(HERE, '..', 'tests'))
import ztamd as zt, zt_oracle
o = zt_oracle.Oracle()
rng = random.Random(4)
files = [o.gen(["wordsalad", "structured", "xorshift32"][i % 3], 9000 + i, rng.randint(1024, 65536)) for i in range(300)]
for f in files[:20]: zt.gzip_compress(f)
t0 = time.perf_counter()
for i, f in enumerate(files): zt.gzip_compress(f, name=b"f%05d" % i, mtime=i)
dt = time.perf_counter() - t0
print(f"{len(files)} files: {1e3*dt/len(files):.3f} ms per call, {len(files)/dt:.0f} files/s", flush=True)
