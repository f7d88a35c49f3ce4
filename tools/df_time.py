# Cycle split of the match kernel per sub-chunk (libzt built with -DZT_DF_TIME, ZT_LIB=...):
# chain build (of which serial linking), search, wait at the barrier after search.
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
    zt.lib.zt_debug_df_time(buf)
    dp.run(d_in.data_ptr(), n, d_c.data_ptr()); torch.cuda.synchronize()
    zt.lib.zt_debug_df_time(buf)
    v = list(buf)
    subs = v[3] & ((1 << 20) - 1)
    link = v[4]
    print(f"{kind:10s} sub-chunks {subs}  cycles/sub: chain_build {v[0]/subs:8.0f} (link {link/subs:8.0f})  search(t0) {v[1]/subs:8.0f}  barrier wait {v[2]/subs:8.0f}", flush=True)
