# Hop statistics of the match kernel (needs libzt built with -DZT_DF_COUNT, ZT_LIB=...)
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
    zt.lib.zt_debug_df_count(buf)
    dp.run(d_in.data_ptr(), n, d_c.data_ptr()); torch.cuda.synchronize()
    zt.lib.zt_debug_df_count(buf)
    v = list(buf)
    print(kind, 'pair-steps/wave', v[0], 'lane hops', v[1], 'extends', v[2], 'hops/position %.2f' % (v[1] / n),
          'lane-util %.2f' % (v[1] / max(1, v[0] * 128)), 'extend passes/step %.2f' % (v[3] / max(1, v[0])),
          'lanes/pass %.1f' % (v[2] / max(1, v[3])),
          'measured: improve %.3f, < 8 bytes %.3f, no gain %.3f' % (v[4] / max(1, v[2]), v[5] / max(1, v[2]),
                                                                v[6] / max(1, v[2])), flush=True)
