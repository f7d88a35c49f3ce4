# Kernel-level single-stream inflate timing through the device plan API.
import sys, time, zlib; sys.path.insert(0,'tests'); sys.path.insert(0,'zlib.ts_amd/py')
import zt_oracle, ztamd, torch
o = zt_oracle.Oracle()
for kind in ["wordsalad", "structured", "xorshift32"]:
    d = o.gen(kind, 7, 4 << 20)
    s = zlib.compress(d, 6)[2:-4]
    di = torch.frombuffer(bytearray(s), dtype=torch.uint8).cuda()
    do = torch.empty(len(d) + 4096, dtype=torch.uint8, device='cuda')
    p = ztamd.InflatePlan(len(s), len(d))
    p.run(di.data_ptr(), len(s), do.data_ptr(), do.numel())
    torch.cuda.synchronize()
    t0 = time.time(); olen, ip = p.run(di.data_ptr(), len(s), do.data_ptr(), do.numel()); dt = time.time() - t0
    assert olen == len(d) and bytes(do[:olen].cpu().numpy()) == d
    print(kind, 'kernel single stream %.1f MB/s, %.1f ms' % (len(d) / dt / 1e6, dt * 1e3), flush=True)
