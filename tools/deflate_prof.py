# Per-phase cycle counters of the deflate kernel (build libzt with -DZT_DF_PROF).
import sys, time, ctypes; sys.path.insert(0, 'zlib.ts_amd/py')
import torch, ztamd
lib = ztamd.lib
buf = (ctypes.c_ulonglong * 8)()
names = ['load', 'chain', 'search', 'parse', 'plan', 'encode']
n = 256 << 20
d = torch.empty(n, dtype=torch.uint8, device='cuda')
c = torch.empty(ztamd.deflate_bound(n), dtype=torch.uint8, device='cuda')
REF = {'wordsalad': 0.15455, 'xorshift32': 1.00075, 'structured': 0.4898}
import os
for level in [int(x) for x in os.environ.get('LEVELS', '6,1').split(',')]:
    p = ztamd.DeflatePlan(n, level=level)
    for kind in ['wordsalad', 'xorshift32', 'structured']:
        ztamd.synth_dev(kind, 3, d.data_ptr(), n)
        p.run(d.data_ptr(), n, c.data_ptr())
        lib.zt_debug_deflate_prof(buf)
        torch.cuda.synchronize()
        t0 = time.time(); clen = p.run(d.data_ptr(), n, c.data_ptr()); dt = time.time() - t0
        lib.zt_debug_deflate_prof(buf)
        v = list(buf)
        mib = n / 2**20
        print(f'L{level} {kind:10s} {n / dt / 2**30:.2f} GiB/s ratio {clen / n:.4f} vs_ref {clen / n / REF[kind]:.4f} | Mcycles per MiB (per WG): ' +
              ' '.join(f'{names[i]}={v[i] / mib / 1e6:.2f}' for i in range(6)), flush=True)
    p.close()
