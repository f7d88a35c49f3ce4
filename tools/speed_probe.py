import sys, time; sys.path.insert(0,'tests'); sys.path.insert(0,'zlib.ts_amd/py')
import zt_oracle, ztamd, torch
o = zt_oracle.Oracle()
N = 256 << 20
parts = []
for i in range(N // (1 << 20)):
    parts.append(o.gen(["wordsalad", "xorshift32", "structured"][i % 3], 100 + i, 1 << 20))
d = b"".join(parts)
t = torch.frombuffer(bytearray(d), dtype=torch.uint8).cuda()
out = torch.empty(ztamd.deflate_bound(N), dtype=torch.uint8, device="cuda")
for lv in (1, 4, 6, 9):
    plan = ztamd.DeflatePlan(N, level=lv)
    n = plan.run(t.data_ptr(), N, out.data_ptr())
    torch.cuda.synchronize()
    ts = []
    for _ in range(3):
        t0 = time.time(); n = plan.run(t.data_ptr(), N, out.data_ptr()); torch.cuda.synchronize(); ts.append(time.time() - t0)
    dt = min(ts)
    print('level', lv, 'ratio %.4f' % (n / N), 'time %.1f ms' % (dt * 1e3), '%.1f GiB/s' % (N / dt / 2**30), flush=True)
    plan.close()
c0 = time.time(); ztamd.dev_checksums(t.data_ptr(), N); torch.cuda.synchronize(); 
c0 = time.time(); ztamd.dev_checksums(t.data_ptr(), N); torch.cuda.synchronize(); print('checksums %.3f ms' % ((time.time()-c0)*1e3))
