# Dump GPU deflate streams for offline analysis (gpurun_out/df_*.bin).
import os, sys; sys.path.insert(0, 'tests'); sys.path.insert(0, 'zlib.ts_amd/py')
import zt_oracle, ztamd as zt
o = zt_oracle.Oracle()
os.makedirs('gpurun_out', exist_ok=True)
for kind, n in [("xorshift32", 65539), ("wordsalad", 65539)]:
    d = o.gen(kind, 1000 + n, n)
    open(f'gpurun_out/df_{kind}_{n}.bin', 'wb').write(zt.deflate_raw(d))
