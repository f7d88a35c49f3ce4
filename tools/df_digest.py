# Deflate output digests and match/pipeline times per corpus (128 MiB) and
# level: two builds (ZT_LIB=...) that must give identical streams print
# identical digests.   usage: [DF_LEVELS=6,1,9] python tools/df_digest.py [kinds...]
import hashlib, os, sys; sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', 'zlib.ts_amd', 'py'))
import torch, ztamd as zt
kinds = sys.argv[1:] or ["wordsalad", "xorshift32", "structured", "mixed"]
n = 128 << 20
d_in = torch.empty(n, dtype=torch.uint8, device="cuda")
d_c = torch.empty(zt.deflate_bound(n), dtype=torch.uint8, device="cuda")
for level in [int(x) for x in os.environ.get("DF_LEVELS", "6,1,9").split(",")]:
    dp = zt.DeflatePlan(n, level=level)
    for kind in kinds:
        zt.synth_dev(kind, 5, d_in.data_ptr(), n)
        clen = dp.run(d_in.data_ptr(), n, d_c.data_ptr())
        zt.timing_enable(True)
        for _ in range(2):
            clen = dp.run(d_in.data_ptr(), n, d_c.data_ptr())
        torch.cuda.synchronize()
        t = zt.timing_read(); zt.timing_enable(False)
        h = hashlib.sha256(d_c[:clen].cpu().numpy().tobytes()).hexdigest()[:16]
        print(f"L{level} {kind:10s} {h} ratio {clen/n:.5f} match {t['deflate_ms']/t['deflate_launches']:6.2f} ms "
              f"pipeline {t['deflate_pipeline_ms']/t['deflate_pipelines']:6.2f} ms", flush=True)
    dp.close()
