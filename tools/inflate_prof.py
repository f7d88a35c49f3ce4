# Per-phase cycle counters of the inflate kernel (build libzt with -DZT_INF_PROF).
import sys, time, zlib, ctypes; sys.path.insert(0,'tests'); sys.path.insert(0,'zlib.ts_amd/py')
import zt_oracle, ztamd, torch
o = zt_oracle.Oracle()
lib = ztamd.lib
buf = (ctypes.c_ulonglong * 16)()
for kind in ["wordsalad", "structured"]:
    d = o.gen(kind, 7, 4 << 20)
    s = zlib.compress(d, 6)[2:-4]
    lib.zt_debug_inflate_prof(buf)
    t0 = time.time(); out, ip = ztamd.inflate_raw(s); dt = time.time() - t0
    lib.zt_debug_inflate_prof(buf)
    v = list(buf)
    print(kind, len(d), len(s), '%.1f MB/s' % (len(d)/dt/1e6), 'lit_dec', v[0], 'lit_store', v[1], 'match_hdr', v[2], 'copy', v[3],
          'kernel', v[4], 'nsym', v[8], 'nmatch', v[9], 'matchbytes', v[10], flush=True)
    if v[8]: print('  cycles/sym decode %.0f, lit store %.0f, match hdr/match %.0f, copy/match %.0f' % (v[0]/v[8], v[1]/max(1,v[8]-v[9]), v[2]/max(1,v[9]), v[3]/max(1,v[9])))
