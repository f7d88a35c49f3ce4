# Cycle split of the match kernel per wave and sub-chunk (libzt built with
# -DZT_DF_TIME, ZT_LIB=...): hash phase, serial link (linker waves), waiting
# for links, searching, idle at the sub-chunk barrier.
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
    ws = v[3]  # (wave, sub-chunk) pairs
    if ws == 0:
        print(f"{kind:10s} no sub-chunk searched (every block stored by classify_kernel)", flush=True)
        continue
    subs = ws / 16
    print(f"{kind:10s} per wave per sub-chunk: hash {v[0]/ws:7.0f}  link(2 waves) {v[4]/subs/2:7.0f}  "
          f"link-wait {v[5]/ws:7.0f}  search {v[1]/ws:7.0f}  loop total {v[7]/ws:7.0f}  barrier idle {v[2]/ws:7.0f}  "
          f"super-steps/wave {v[6]/ws:5.2f}", flush=True)
