"""The C-ABI boundary (include/*.h): libzt.so loads without a GPU, exports
every function the headers declare, and refuses to compute without a GPU
(there is no CPU fallback)."""
import ctypes
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "zt.h")


def declared_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    names = set(re.findall(r"\b(zt_[a-z0-9_]+)\s*\(", text))
    return sorted(names)


def test_header_declares_the_boundary():
    names = declared_functions()
    for want in ["zt_crc32_update", "zt_adler32_update", "zt_deflate_raw", "zt_inflate_raw",
                 "zt_deflate_raw_batch", "zt_inflate_raw_batch", "zt_device_count", "zt_last_error_message"]:
        assert want in names


def test_library_exports_every_declared_symbol():
    import ztamd

    lib = ctypes.CDLL(ztamd.LIBPATH)
    missing = [n for n in declared_functions() if not hasattr(lib, n)]
    assert not missing, missing
    assert sorted(ztamd.SYMBOLS) == declared_functions()


def test_no_cpu_fallback_without_gpu():
    import torch
    import ztamd

    if torch.cuda.is_available():
        return  # the GPU suite covers the compute path
    assert ztamd.device_count() == 0
    for call in (lambda: ztamd.crc32(b"123456789"), lambda: ztamd.deflate_raw(b"abc"),
                 lambda: ztamd.inflate_raw(b"\x03\x00")):
        try:
            call()
        except ztamd.ZtError as e:
            assert e.code == -100  # ZT_E_NO_DEVICE
        else:
            raise AssertionError("computed without a GPU")
