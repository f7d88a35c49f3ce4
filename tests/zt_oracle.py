"""ctypes view of oracle/liboracle.so -- TEST INFRASTRUCTURE ONLY.

The oracle is the CPU restatement of the reference (oracle/zt_oracle.c).  It is
loaded only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg,
as the checker; the product never routes through it.
"""
import ctypes
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "oracle", "liboracle.so")

ERR_INFLATE = -10
KINDS = {"xorshift32": 0, "wordsalad": 1, "structured": 2}


def _load():
    if not os.path.exists(LIB):
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle")])
    lib = ctypes.CDLL(LIB)
    u8p = ctypes.POINTER(ctypes.c_uint8)
    sz = ctypes.c_size_t
    lib.zo_crc32_update.restype = ctypes.c_uint32
    lib.zo_crc32_update.argtypes = [ctypes.c_void_p, sz, ctypes.c_uint32]
    lib.zo_crc32_single.restype = ctypes.c_uint32
    lib.zo_crc32_single.argtypes = [ctypes.c_uint32, ctypes.c_uint32]
    lib.zo_adler32_update.restype = ctypes.c_uint32
    lib.zo_adler32_update.argtypes = [ctypes.c_uint32, ctypes.c_void_p, sz]
    lib.zo_raw_deflate.restype = ctypes.c_int
    lib.zo_raw_deflate.argtypes = [ctypes.c_void_p, sz, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, sz, sz,
                                   ctypes.POINTER(u8p), ctypes.POINTER(sz), ctypes.POINTER(sz)]
    lib.zo_raw_inflate.restype = ctypes.c_int
    lib.zo_raw_inflate.argtypes = [ctypes.c_void_p, sz, sz, ctypes.c_int, sz, ctypes.POINTER(u8p),
                                   ctypes.POINTER(sz), ctypes.POINTER(sz), ctypes.c_char_p, sz]
    lib.zo_gen.restype = None
    lib.zo_gen.argtypes = [ctypes.c_int, ctypes.c_uint32, ctypes.c_void_p, sz]
    lib.zo_free.argtypes = [ctypes.c_void_p]
    lib.zo_huffman_lengths.argtypes = [ctypes.POINTER(ctypes.c_uint32), sz, ctypes.c_int, u8p]
    return lib


def _buf(data):
    data = bytes(data)
    return ctypes.create_string_buffer(data, len(data) or 1), len(data)


class OracleError(Exception):
    def __init__(self, code, msg=""):
        super().__init__(msg or f"oracle status {code}")
        self.code = code
        self.msg = msg


class Oracle:
    def __init__(self):
        self.lib = _load()

    def crc32(self, data, crc=0):
        b, n = _buf(data)
        return self.lib.zo_crc32_update(b, n, crc)

    def crc32_single(self, num, crc):
        return self.lib.zo_crc32_single(num, crc)

    def adler32(self, data, adler=1):
        b, n = _buf(data)
        return self.lib.zo_adler32_update(adler, b, n)

    def raw_deflate(self, data, lazy=0, ctype=2, outbuf=None, out_index=0):
        b, n = _buf(data)
        ob, obn = (None, 0) if outbuf is None else _buf(outbuf)
        if outbuf is not None:
            obn = len(outbuf)
        out = ctypes.POINTER(ctypes.c_uint8)()
        olen = ctypes.c_size_t()
        op = ctypes.c_size_t()
        rc = self.lib.zo_raw_deflate(b, n, lazy, ctype, ob, obn, out_index, ctypes.byref(out), ctypes.byref(olen),
                                     ctypes.byref(op))
        if rc:
            raise OracleError(rc)
        res = ctypes.string_at(out, olen.value)
        self.lib.zo_free(out)
        return res, op.value

    def raw_inflate(self, data, index=0, buffer_type=1, buffer_size=0x8000):
        b, n = _buf(data)
        out = ctypes.POINTER(ctypes.c_uint8)()
        olen = ctypes.c_size_t()
        ip = ctypes.c_size_t()
        msg = ctypes.create_string_buffer(256)
        rc = self.lib.zo_raw_inflate(b, n, index, buffer_type, buffer_size, ctypes.byref(out), ctypes.byref(olen),
                                     ctypes.byref(ip), msg, 256)
        if rc:
            raise OracleError(rc, msg.value.decode())
        res = ctypes.string_at(out, olen.value)
        self.lib.zo_free(out)
        return res, ip.value

    def gen(self, kind, seed, n):
        buf = ctypes.create_string_buffer(n or 1)
        self.lib.zo_gen(KINDS[kind], seed, buf, n)
        return buf.raw[:n]
