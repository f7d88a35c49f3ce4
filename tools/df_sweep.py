# Ratio / match-kernel time for deflate parameter sets (ZT_DF_PARAMS) on a corpus.
import os, sys; sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', 'zlib.ts_amd', 'py'))
import torch, ztamd as zt
kind = sys.argv[1]
n = 128 << 20
d_in = torch.empty(n, dtype=torch.uint8, device="cuda")
zt.synth_dev(kind, 5, d_in.data_ptr(), n)
d_c = torch.empty(zt.deflate_bound(n), dtype=torch.uint8, device="cuda")
dp = zt.DeflatePlan(n)
for ps in sys.argv[2:]:
    os.environ["ZT_DF_PARAMS"] = ps
    clen = dp.run(d_in.data_ptr(), n, d_c.data_ptr())
    zt.timing_enable(True)
    for _ in range(2):
        clen = dp.run(d_in.data_ptr(), n, d_c.data_ptr())
    torch.cuda.synchronize()
    t = zt.timing_read(); zt.timing_enable(False)
    print(f"{kind:10s} {ps:28s} ratio {clen/n:.4f} match {t['deflate_ms']/t['deflate_launches']:6.2f} ms  pipeline {t['deflate_pipeline_ms']/t['deflate_pipelines']:6.2f} ms", flush=True)
