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

    # ---- containers: host byte logic restated in
    # Python over the C oracle's RawInflate / CRC32 / Adler32 ----------------
    @staticmethod
    def header_bytes(s):
        """String -> header bytes as src/GZip.ts:133-150 writes them: a char
        code <= 0xFF is one byte, anything wider two little-endian bytes."""
        out = bytearray()
        for ch in s:
            c = ord(ch)
            out += bytes([c & 0xFF, (c >> 8) & 0xFF]) if c > 0xFF else bytes([c])
        return bytes(out)

    def gzip_header(self, name=None, comment=None, hcrc=False, mtime=0):
        """src/GZip.ts:104-156 (header up to the DEFLATE stream)."""
        flg = (0x08 if name is not None else 0) | (0x10 if comment is not None else 0) | (0x02 if hcrc else 0)
        h = bytearray([0x1F, 0x8B, 8, flg]) + mtime.to_bytes(4, "little") + bytes([0, 3])
        if name is not None:
            h += name + b"\0"
        if comment is not None:
            h += comment + b"\0"
        if hcrc:
            h += (self.crc32(bytes(h)) & 0xFFFF).to_bytes(2, "little")
        return bytes(h)

    def gunzip(self, data):
        """src/GUnzip.ts:53-175: members until the input is consumed.  Bytes
        read past the end are `undefined` (0 inside bitwise expressions).
        Returns (output, members); raises OracleError(msg=reference text)."""
        n = len(data)
        u8 = lambda p: data[p] if p < n else 0
        ip, members = 0, []
        while ip < n:
            p = ip
            if u8(p) != 0x1F or u8(p + 1) != 0x8B:
                a = str(data[p]) if p < n else "undefined"
                b = str(data[p + 1]) if p + 1 < n else "undefined"
                raise OracleError(-30, f"invalid file signature:{a},{b}")
            if p + 2 >= n or data[p + 2] != 8:
                raise OracleError(-31, "unknown compression method: " + (str(data[p + 2]) if p + 2 < n else "undefined"))
            flg = u8(p + 3)
            m = {"flg": flg, "mtime": int.from_bytes(bytes(u8(p + 4 + k) for k in range(4)), "little"),
                 "xfl": u8(p + 8), "os": u8(p + 9), "name": None, "comment": None}
            p += 10
            if flg & 0x04:
                p += 2 + (u8(p) | (u8(p + 1) << 8))
            for bit, key in ((0x08, "name"), (0x10, "comment")):
                if flg & bit:
                    e = data.find(b"\0", p)
                    e = n if e < 0 else e
                    m[key] = data[p:e]
                    p = e + 1
            if flg & 0x02:
                c16 = self.crc32(data[:p]) & 0xFFFF
                if c16 != (u8(p) | (u8(p + 1) << 8)):
                    raise OracleError(-32, "invalid header crc16")
                p += 2
            try:
                out, eip = self.raw_inflate(data, index=p)
            except OracleError as e:
                raise OracleError(e.code, e.msg)
            want = int.from_bytes(bytes(u8(eip + k) for k in range(4)), "little")
            crc = self.crc32(out)
            if crc != want:
                raise OracleError(-33, "invalid CRC-32 checksum: 0x%x / 0x%x" % (crc, want))
            isize = int.from_bytes(bytes(u8(eip + 4 + k) for k in range(4)), "little")
            if len(out) & 0xFFFFFFFF != isize:
                raise OracleError(-34, "invalid input size: %d / %d" % (len(out) & 0xFFFFFFFF, isize))
            m["data"] = out
            m["crc32"] = crc
            members.append(m)
            ip = eip + 8
        return b"".join(m["data"] for m in members), members

    def zlib_header(self, compression_type=2):
        """src/Deflate.ts:67-78: CMF 0x78, FLG with FLEVEL = compressionType."""
        flg = compression_type << 6
        return bytes([0x78, flg | (31 - ((0x78 << 8) + flg) % 31)])

    def zlib_inflate(self, data, index=0, verify=False):
        """src/Inflate.ts:34-93.  Returns (output, ip)."""
        n = len(data)
        cmf = data[index] if index < n else None
        flg = data[index + 1] if index + 1 < n else None
        if cmf is None or (cmf & 0x0F) != 8:
            raise OracleError(-40, "unsupported compression method")
        if flg is None:
            raise OracleError(-41, "invalid fcheck flag:NaN")
        if ((cmf << 8) + flg) % 31:
            raise OracleError(-41, "invalid fcheck flag:%d" % (((cmf << 8) + flg) % 31))
        if flg & 0x20:
            raise OracleError(-42, "fdict flag is not supported")
        out, ip = self.raw_inflate(data, index=index + 2)
        if verify:
            want = int.from_bytes(bytes(data[ip + k] if ip + k < n else 0 for k in range(4)), "big")
            if self.adler32(out) != want:
                raise OracleError(-43, "invalid adler-32 checksum")
        return out, ip
