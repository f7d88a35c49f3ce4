# Cycle split of block_kernel phases (libzt built with -DZT_DF_TIME, ZT_LIB=...).
import ctypes, os, sys; sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', 'zlib.ts_amd', 'py'))
import torch, ztamd as zt
buf = (ctypes.c_ulonglong * 8)()
for kind in sys.argv[1:]:
    n = 128 << 20
    d_in = torch.empty(n, dtype=torch.uint8, device="cuda")
    zt.synth_dev(kind, 5, d_in.data_ptr(), n)
    d_c = torch.empty(zt.deflate_bound(n), dtype=torch.uint8, device="cuda")
    dp = zt.DeflatePlan(n)
    dp.run(d_in.data_ptr(), n, d_c.data_ptr()); torch.cuda.synchronize()
    zt.lib.zt_debug_bk_time(buf)
    dp.run(d_in.data_ptr(), n, d_c.data_ptr()); torch.cuda.synchronize()
    zt.lib.zt_debug_bk_time(buf)
    v = list(buf); nb = max(1, v[6])
    names = ['parse', 'huff lit+dist', 'rle', 'cl huff+codes', 'sizes', 'plan+header']
    print(f"{kind:10s} blocks {nb}  cycles/block: " + '  '.join(f"{nm} {v[i]/nb:7.0f}" for i, nm in enumerate(names)), flush=True)
