"""Config C4 at its own workload: GZip end-to-end of the
10 000-file batch (tests/c4_corpus.py, ~1.41 GiB, half text / half binary)
through ONE zt_gzip_compress_batch call (src/GZip.ts:96-194 per file: header,
RawDeflate, CRC-32 + ISIZE trailer).  Every member's header, CRC-32 and ISIZE
are checked, every member is decoded by Python's zlib and by the engine's
GUnzip (src/GUnzip.ts:53-175, multi-member), and a fixed sample of 220 by the
oracle's RawInflate (the reference's algorithm, pinned by tests/golden).  The
same batch spread over 8 logical devices (ZT_ALIAS_DEVICES=8) must give
byte-identical members."""
import json
import os
import random
import subprocess
import sys
import time
import zlib

import pytest

from c4_corpus import FILES, c4_files, members_digest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def zt():
    import ztamd

    assert ztamd.device_count() > 0, "no GPU visible"
    return ztamd


@pytest.fixture(scope="module")
def c4(zt, oracle):
    files = c4_files(oracle)
    total = sum(len(f) for f in files)
    assert len(files) == FILES and 1.3 * 2**30 < total < 1.55 * 2**30, total
    best, members = None, None
    for _ in range(2):
        t0 = time.perf_counter()
        m = zt.gzip_compress_batch(files, mtime=0)
        dt = time.perf_counter() - t0
        members = members if members is not None else m
        assert m == members  # deterministic
        best = dt if best is None else min(best, dt)
    comp = sum(len(x) for x in members)
    rec = {"files": FILES, "bytes": total, "seconds": round(best, 4), "GiBps": round(total / best / 2**30, 3),
           "files_per_s": round(FILES / best, 1), "ratio": round(comp / total, 5)}
    print("C4", json.dumps(rec), flush=True)
    out = os.environ.get("ZT_C4_RECORD")
    if out:
        with open(out, "w") as fh:
            json.dump(rec, fh, indent=1)
    return files, members


def test_c4_members_header_trailer_zlib(c4, oracle):
    files, members = c4
    head = oracle.gzip_header()
    assert len(members) == len(files)
    for f, m in zip(files, members):
        assert m[:len(head)] == head
        assert m[-8:-4] == zlib.crc32(f).to_bytes(4, "little")
        assert m[-4:] == (len(f) & 0xFFFFFFFF).to_bytes(4, "little")
        assert zlib.decompress(m, 31) == f


def test_c4_engine_gunzip(zt, c4):
    files, members = c4
    step = 500
    for a in range(0, len(files), step):
        out, mem = zt.gunzip(b"".join(members[a:a + step]))
        assert len(mem) == len(members[a:a + step])
        assert out == b"".join(files[a:a + step])


def test_c4_oracle_sample(c4, oracle):
    files, members = c4
    order = sorted(range(len(files)), key=lambda i: len(files[i]))
    sample = sorted(set(random.Random(5).sample(range(len(files)), 200) + order[:10] + order[-10:]))
    assert len(sample) >= 200
    for i in sample:
        body, ip = oracle.raw_inflate(members[i], index=10)
        assert body == files[i]
        assert members[i][ip:ip + 4] == oracle.crc32(files[i]).to_bytes(4, "little")
        assert ip + 8 == len(members[i])


def test_c4_alias_devices(c4):
    """The same batch over 8 logical devices (LPT split, one host thread per
    device): byte-identical members."""
    files, members = c4
    here = os.path.dirname(os.path.abspath(__file__))
    env = dict(os.environ, ZT_ALIAS_DEVICES="8")
    p = subprocess.run([sys.executable, os.path.join(here, "c4_alias_child.py")], env=env, capture_output=True,
                       text=True, timeout=110)
    assert p.returncode == 0, p.stderr[-2000:]
    res = json.loads(p.stdout.strip().splitlines()[-1])
    assert res == {"logical_devices": 8, "members": len(members), "digest": members_digest(members)}, res
