"""Host entry points called from several threads at once on one device: the
per-device lock (DeviceCtx::mu) serialises their use of the shared scratch,
pinned staging and streams, so every call's result is the single-threaded
one.  ctypes releases the GIL inside the calls, so the threads really run
concurrently."""
import threading
import zlib

import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def zt():
    import ztamd

    assert ztamd.device_count() > 0, "no GPU visible"
    return ztamd


def test_threads_share_device(zt, oracle):
    kinds = ["wordsalad", "structured", "xorshift32"]
    data = [oracle.gen(kinds[i % 3], 3000 + i, 20000 + 7919 * i) for i in range(8)]
    errors = []

    def work(t):
        try:
            for r in range(4):
                d = data[(t + r) % len(data)]
                s = zt.deflate_raw(d, level=6)
                out, ip = zt.inflate_raw(s)
                assert out == d and ip == len(s)
                g, crc = zt.gzip_compress(d)
                assert crc == zlib.crc32(d)
                assert zlib.decompress(g, 31) == d
                res = zt.inflate_raw_batch([zlib.compress(x, 6)[2:-4] for x in data])
                assert all(st == 0 and o == x for (st, o, _), x in zip(res, data))
        except Exception as e:  # reported in the main thread
            errors.append(f"thread {t}: {e!r}")

    th = [threading.Thread(target=work, args=(t,)) for t in range(4)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    assert not errors, errors
