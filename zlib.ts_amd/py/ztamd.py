"""ztamd -- ctypes binding of libzt.so (include/zt.h) for tests and bench.py.

This is plumbing over the C-ABI, not a second implementation: every call runs
on the GPU through libzt.so.  Importing fails loudly when the library has not
been built (``make -C zlib.ts_amd`` / ``__graft_entry__.build()``).
"""
import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIBPATH = os.environ.get("ZT_LIB") or os.path.join(os.path.dirname(HERE), "libzt.so")

ZT_OK = 0
ERRORS = {
    -1: "ZT_E_INVALID_COMPRESSION_TYPE", -2: "ZT_E_INVALID_INDEX", -10: "ZT_E_INPUT_BROKEN",
    -11: "ZT_E_INVALID_CODE_LENGTH", -12: "ZT_E_UNKNOWN_BTYPE", -13: "ZT_E_STORED_LEN", -14: "ZT_E_STORED_NLEN",
    -15: "ZT_E_INVALID_DISTANCE", -16: "ZT_E_INVALID_SYMBOL", -17: "ZT_E_BAD_TREE",
    -30: "ZT_E_GZIP_SIGNATURE", -31: "ZT_E_GZIP_METHOD", -32: "ZT_E_GZIP_HCRC", -33: "ZT_E_GZIP_CRC32",
    -34: "ZT_E_GZIP_ISIZE", -40: "ZT_E_ZLIB_METHOD", -41: "ZT_E_ZLIB_FCHECK", -42: "ZT_E_ZLIB_FDICT",
    -43: "ZT_E_ZLIB_ADLER", -100: "ZT_E_NO_DEVICE",
    -101: "ZT_E_HIP", -102: "ZT_E_NOMEM", -103: "ZT_E_ARG", -104: "ZT_E_INTERNAL",
}


class ZtError(Exception):
    def __init__(self, code, msg):
        super().__init__(f"{ERRORS.get(code, code)}: {msg}")
        self.code = code
        self.msg = msg


class DeflateOpts(ctypes.Structure):
    _fields_ = [("compression_type", ctypes.c_int), ("lazy", ctypes.c_int), ("level", ctypes.c_int)]


class KernelTimes(ctypes.Structure):
    _fields_ = [("deflate_ms", ctypes.c_double), ("deflate_launches", ctypes.c_uint64),
                ("inflate_ms", ctypes.c_double), ("inflate_launches", ctypes.c_uint64),
                ("deflate_pipeline_ms", ctypes.c_double), ("deflate_pipelines", ctypes.c_uint64),
                ("inflate_tok_ms", ctypes.c_double), ("inflate_toks", ctypes.c_uint64),
                ("inflate_paths", ctypes.c_uint64 * 3), ("general_passes", ctypes.c_uint64),
                ("blocks_unsearched", ctypes.c_uint64)]


class ZipFile(ctypes.Structure):
    _fields_ = [("name", ctypes.c_char_p), ("name_len", ctypes.c_size_t), ("comment", ctypes.c_char_p),
                ("comment_len", ctypes.c_size_t), ("method", ctypes.c_int), ("os", ctypes.c_int),
                ("mtime", ctypes.c_uint8 * 4), ("deflate", DeflateOpts)]


class UnzipEntry(ctypes.Structure):
    _fields_ = [("name_off", ctypes.c_size_t), ("name_len", ctypes.c_size_t), ("comment_off", ctypes.c_size_t),
                ("comment_len", ctypes.c_size_t), ("data_off", ctypes.c_size_t), ("data_len", ctypes.c_size_t),
                ("local_offset", ctypes.c_size_t)] + [
                    (f, ctypes.c_uint32) for f in ("version", "os", "need_version", "flags", "method", "time", "date",
                                                   "crc32", "compressed_size", "plain_size", "local_crc32",
                                                   "local_method", "data_crc32")] + [
                    ("status", ctypes.c_int32), ("message", ctypes.c_char * 96)]


class InflateOpts(ctypes.Structure):
    _fields_ = [("buffer_type", ctypes.c_int), ("buffer_size", ctypes.c_size_t), ("ref_strict", ctypes.c_int)]


class GzipOpts(ctypes.Structure):
    _fields_ = [("deflate", DeflateOpts), ("fname", ctypes.c_int), ("fcomment", ctypes.c_int),
                ("fhcrc", ctypes.c_int), ("mtime", ctypes.c_uint32), ("name", ctypes.c_char_p),
                ("name_len", ctypes.c_size_t), ("comment", ctypes.c_char_p), ("comment_len", ctypes.c_size_t)]


class GzipMember(ctypes.Structure):
    _fields_ = [("flg", ctypes.c_uint32), ("mtime", ctypes.c_uint32), ("xfl", ctypes.c_uint32),
                ("os", ctypes.c_uint32), ("xlen", ctypes.c_uint32), ("name_off", ctypes.c_size_t),
                ("name_len", ctypes.c_size_t), ("comment_off", ctypes.c_size_t), ("comment_len", ctypes.c_size_t),
                ("has_crc16", ctypes.c_uint32), ("crc16", ctypes.c_uint32), ("crc32", ctypes.c_uint32),
                ("isize", ctypes.c_uint32), ("data_off", ctypes.c_size_t), ("data_len", ctypes.c_size_t)]


def _load():
    # torch (when present) ships its own libamdhip64.so.7; loading it first makes
    # libzt.so bind to that same runtime (same SONAME) instead of starting a
    # second HIP runtime in the process, which would leave torch without a GPU.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    if not os.path.exists(LIBPATH):
        raise ImportError(f"libzt.so not built at {LIBPATH}; run make -C zlib.ts_amd")
    lib = ctypes.CDLL(LIBPATH)
    sz, vp, u32 = ctypes.c_size_t, ctypes.c_void_p, ctypes.c_uint32
    u8pp = ctypes.POINTER(ctypes.POINTER(ctypes.c_uint8))
    P = ctypes.POINTER
    sig = {
        "zt_device_count": ([], ctypes.c_int),
        "zt_set_device": ([ctypes.c_int], ctypes.c_int),
        "zt_set_devices": ([ctypes.c_uint64], ctypes.c_int),
        "zt_last_error_message": ([], ctypes.c_char_p),
        "zt_version": ([], ctypes.c_char_p),
        "zt_free": ([vp], None),
        "zt_crc32_update": ([u32, vp, sz, P(u32)], ctypes.c_int),
        "zt_adler32_update": ([u32, vp, sz, P(u32)], ctypes.c_int),
        "zt_checksums": ([vp, sz, u32, u32, P(u32), P(u32)], ctypes.c_int),
        "zt_deflate_raw": ([vp, sz, P(DeflateOpts), u8pp, P(sz)], ctypes.c_int),
        "zt_inflate_raw": ([vp, sz, sz, P(InflateOpts), u8pp, P(sz), P(sz)], ctypes.c_int),
        "zt_inflate_raw_resume": ([vp, sz, ctypes.c_uint64, vp, sz, u8pp, P(sz), P(ctypes.c_uint64),
                                   P(ctypes.c_int)], ctypes.c_int),
        "zt_inflate_raw_resume_final": ([vp, sz, ctypes.c_uint64, vp, sz, u8pp, P(sz), P(ctypes.c_uint64),
                                         P(ctypes.c_int)], ctypes.c_int),
        "zt_inflate_raw_batch": ([P(vp), P(sz), sz, P(InflateOpts), u8pp, P(sz), P(sz), P(ctypes.c_int)],
                                 ctypes.c_int),
        "zt_deflate_raw_batch": ([P(vp), P(sz), sz, P(DeflateOpts), u8pp, P(sz), P(ctypes.c_int)], ctypes.c_int),
        "zt_gzip_compress": ([vp, sz, P(GzipOpts), u8pp, P(sz), P(u32)], ctypes.c_int),
        "zt_gzip_compress_batch": ([P(vp), P(sz), sz, P(GzipOpts), u8pp, P(sz), P(ctypes.c_int)], ctypes.c_int),
        "zt_zlib_compress_batch": ([P(vp), P(sz), sz, P(DeflateOpts), u8pp, P(sz), P(ctypes.c_int)], ctypes.c_int),
        "zt_crc32_batch": ([P(vp), P(sz), sz, P(u32)], ctypes.c_int),
        "zt_zip_compress": ([P(vp), P(sz), P(ZipFile), sz, vp, sz, u8pp, P(sz)], ctypes.c_int),
        "zt_unzip": ([vp, sz, ctypes.c_int, u8pp, P(sz), P(P(UnzipEntry)), P(sz)], ctypes.c_int),
        "zt_gunzip": ([vp, sz, u8pp, P(sz), P(P(GzipMember)), P(sz)], ctypes.c_int),
        "zt_zlib_compress": ([vp, sz, P(DeflateOpts), u8pp, P(sz), P(u32)], ctypes.c_int),
        "zt_zlib_decompress": ([vp, sz, sz, ctypes.c_int, u8pp, P(sz), P(sz), P(u32)], ctypes.c_int),
        "zt_dev_checksums": ([vp, sz, u32, u32, P(u32), P(u32), vp], ctypes.c_int),
        "zt_deflate_plan_create": ([sz, P(DeflateOpts), P(vp)], ctypes.c_int),
        "zt_deflate_plan_destroy": ([vp], None),
        "zt_deflate_bound": ([sz], sz),
        "zt_deflate_dev": ([vp, vp, sz, sz, ctypes.c_int, vp, P(sz), vp], ctypes.c_int),
        "zt_inflate_plan_create": ([sz, sz, P(vp)], ctypes.c_int),
        "zt_inflate_plan_destroy": ([vp], None),
        "zt_inflate_dev": ([vp, vp, sz, vp, sz, P(sz), P(sz), vp], ctypes.c_int),
        "zt_synth_dev": ([ctypes.c_int, u32, vp, sz, vp], ctypes.c_int),
        "zt_synth_dev_at": ([ctypes.c_int, u32, ctypes.c_uint64, vp, sz, vp], ctypes.c_int),
        "zt_timing_enable": ([ctypes.c_int], ctypes.c_int),
        "zt_timing_read": ([P(KernelTimes)], ctypes.c_int),
        "zt_scratch_bytes": ([P(sz), P(sz)], ctypes.c_int),
        "zt_release_scratch": ([], ctypes.c_int),
    }
    for name, (args, res) in sig.items():
        f = getattr(lib, name, None)
        if f is None:  # reported by tests/test_abi.py
            continue
        f.argtypes = args
        f.restype = res
    return lib


lib = _load()

# every symbol include/zt.h declares (checked by tests/test_abi.py)
SYMBOLS = [
    "zt_device_count", "zt_set_device", "zt_set_devices", "zt_last_error_message", "zt_version", "zt_free", "zt_crc32_update",
    "zt_adler32_update", "zt_checksums", "zt_deflate_raw", "zt_inflate_raw", "zt_inflate_raw_resume", "zt_inflate_raw_resume_final",
    "zt_inflate_raw_batch",
    "zt_deflate_raw_batch", "zt_gzip_compress", "zt_gzip_compress_batch", "zt_zlib_compress_batch", "zt_gunzip",
    "zt_crc32_batch", "zt_zip_compress", "zt_unzip", "zt_zlib_compress", "zt_zlib_decompress",
    "zt_dev_checksums", "zt_deflate_plan_create", "zt_deflate_plan_destroy",
    "zt_deflate_bound", "zt_deflate_dev", "zt_inflate_plan_create", "zt_inflate_plan_destroy", "zt_inflate_dev",
    "zt_synth_dev", "zt_synth_dev_at", "zt_timing_enable", "zt_timing_read", "zt_scratch_bytes",
    "zt_release_scratch",
]


def _check(rc):
    if rc != ZT_OK:
        raise ZtError(rc, lib.zt_last_error_message().decode(errors="replace"))


def _cbuf(data):
    data = bytes(data)
    return ctypes.create_string_buffer(data, len(data) or 1), len(data)


def device_count():
    return lib.zt_device_count()


def set_devices(mask):
    """Devices the batch calls split over (bit d = device d; 0 = this thread's)."""
    _check(lib.zt_set_devices(mask))


def set_device(d):
    _check(lib.zt_set_device(d))


def crc32(data, crc=0):
    b, n = _cbuf(data)
    out = ctypes.c_uint32()
    _check(lib.zt_crc32_update(crc, b, n, ctypes.byref(out)))
    return out.value


def adler32(data, adler=1):
    b, n = _cbuf(data)
    out = ctypes.c_uint32()
    _check(lib.zt_adler32_update(adler, b, n, ctypes.byref(out)))
    return out.value


def checksums(data, crc=0, adler=1):
    b, n = _cbuf(data)
    c, a = ctypes.c_uint32(), ctypes.c_uint32()
    _check(lib.zt_checksums(b, n, crc, adler, ctypes.byref(c), ctypes.byref(a)))
    return c.value, a.value


def deflate_raw(data, compression_type=2, lazy=0, level=-1):
    b, n = _cbuf(data)
    opts = DeflateOpts(compression_type, lazy, level)
    out = ctypes.POINTER(ctypes.c_uint8)()
    olen = ctypes.c_size_t()
    _check(lib.zt_deflate_raw(b, n, ctypes.byref(opts), ctypes.byref(out), ctypes.byref(olen)))
    res = ctypes.string_at(out, olen.value)
    lib.zt_free(out)
    return res


def inflate_raw(data, index=0, ref_strict=False, buffer_type=1, buffer_size=0x8000):
    """Returns (output bytes, end ip)."""
    b, n = _cbuf(data)
    opts = InflateOpts(buffer_type, buffer_size, 1 if ref_strict else 0)
    out = ctypes.POINTER(ctypes.c_uint8)()
    olen = ctypes.c_size_t()
    ip = ctypes.c_size_t()
    _check(lib.zt_inflate_raw(b, n, index, ctypes.byref(opts), ctypes.byref(out), ctypes.byref(olen),
                              ctypes.byref(ip)))
    res = ctypes.string_at(out, olen.value)
    lib.zt_free(out)
    return res, ip.value


def inflate_raw_resume(data, bit_pos=0, window=b"", final=False):
    """zt_inflate_raw_resume (final: zt_inflate_raw_resume_final -- no more
    input will come, errors are the stream's own): (output of the complete
    blocks, end bit, finished)."""
    b, n = _cbuf(data)
    w, wn = _cbuf(window)
    out = ctypes.POINTER(ctypes.c_uint8)()
    olen = ctypes.c_size_t()
    end = ctypes.c_uint64()
    fin = ctypes.c_int()
    fn = lib.zt_inflate_raw_resume_final if final else lib.zt_inflate_raw_resume
    _check(fn(b, n, bit_pos, w, wn, ctypes.byref(out), ctypes.byref(olen), ctypes.byref(end), ctypes.byref(fin)))
    res = ctypes.string_at(out, olen.value) if out else b""
    if out:
        lib.zt_free(out)
    return res, end.value, bool(fin.value)


class RawInflateStream:
    """The reference's streaming decoder surface (src/RawInflateStream.ts:
    52-120): ``decompress(new_input, ip)`` decodes what the input holds so far
    and returns the bytes produced by this call.  State between calls: the
    input position (byte ``ip`` and the bits of it already used), the last 32
    KiB of output (match history) and whether the final block was seen."""

    def __init__(self, data=b"", ip=0):
        self.input = bytes(data)
        self.ip = ip
        self.bit = 0
        self.window = b""
        self.bfinal = False
        self.total = 0

    def decompress(self, new_input=None, ip=None):
        return self._run(new_input, ip, False)

    def finish(self, new_input=None, ip=None):
        """The input is complete: decode what is left; a stream corrupt near
        its end, or one that ends before its final block, raises ZtError."""
        out = self._run(new_input, ip, True)
        if not self.bfinal:
            raise ZtError(-10, "input buffer is broken")
        return out

    def _run(self, new_input, ip, final):
        if new_input is not None:
            self.input = bytes(new_input)
        if ip is not None:  # (a re-based buffer: the bits of its byte `ip` already used stay used)
            self.ip = ip
        if self.bfinal or (self.ip >= len(self.input) and not final):
            return b""
        out, end, fin = inflate_raw_resume(self.input, self.ip * 8 + self.bit, self.window, final)
        self.ip, self.bit = end >> 3, end & 7
        self.bfinal = fin
        self.total += len(out)
        self.window = (self.window + out)[-32768:]
        return out


def inflate_raw_batch(streams, ref_strict=False):
    """Returns a list of (status, output bytes, end ip)."""
    k = len(streams)
    # the bytes objects' own buffers are passed (no copy); `bs` keeps them alive
    bs = [bytes(x) for x in streams]
    ptrs = (ctypes.c_void_p * k)(*[ctypes.cast(ctypes.c_char_p(x), ctypes.c_void_p).value for x in bs])
    lens = (ctypes.c_size_t * k)(*[len(x) for x in bs])
    outs = (ctypes.POINTER(ctypes.c_uint8) * k)()
    olens = (ctypes.c_size_t * k)()
    ips = (ctypes.c_size_t * k)()
    st = (ctypes.c_int * k)()
    opts = InflateOpts(1, 0x8000, 1 if ref_strict else 0)
    rc = lib.zt_inflate_raw_batch(ptrs, lens, k, ctypes.byref(opts), outs, olens, ips, st)
    if rc != ZT_OK and all(s == 0 for s in st):
        _check(rc)
    res = []
    for i in range(k):
        data = ctypes.string_at(outs[i], olens[i]) if st[i] == 0 and outs[i] else b""
        if outs[i]:
            lib.zt_free(outs[i])
        res.append((st[i], data, ips[i]))
    return res


def deflate_raw_batch(items, compression_type=2, level=-1):
    k = len(items)
    bufs = [_cbuf(s) for s in items]
    ptrs = (ctypes.c_void_p * k)(*[ctypes.addressof(b) for b, _ in bufs])
    lens = (ctypes.c_size_t * k)(*[n for _, n in bufs])
    outs = (ctypes.POINTER(ctypes.c_uint8) * k)()
    olens = (ctypes.c_size_t * k)()
    st = (ctypes.c_int * k)()
    opts = DeflateOpts(compression_type, 0, level)
    rc = lib.zt_deflate_raw_batch(ptrs, lens, k, ctypes.byref(opts), outs, olens, st)
    _check(rc)
    res = []
    for i in range(k):
        res.append(ctypes.string_at(outs[i], olens[i]))
        lib.zt_free(outs[i])
    return res


def _take(out, olen):
    res = ctypes.string_at(out, olen.value)
    lib.zt_free(out)
    return res


def gzip_compress(data, name=None, comment=None, hcrc=False, mtime=0, compression_type=2, lazy=0, level=-1):
    """GZip.compress (src/GZip.ts:96-194); name/comment are header bytes.
    Returns (member bytes, crc32)."""
    b, n = _cbuf(data)
    o = GzipOpts()
    o.deflate = DeflateOpts(compression_type, lazy, level)
    o.fname, o.fcomment, o.fhcrc, o.mtime = int(name is not None), int(comment is not None), int(hcrc), mtime
    if name is not None:
        o.name, o.name_len = bytes(name), len(name)
    if comment is not None:
        o.comment, o.comment_len = bytes(comment), len(comment)
    out = ctypes.POINTER(ctypes.c_uint8)()
    olen = ctypes.c_size_t()
    crc = ctypes.c_uint32()
    _check(lib.zt_gzip_compress(b, n, ctypes.byref(o), ctypes.byref(out), ctypes.byref(olen), ctypes.byref(crc)))
    return _take(out, olen), crc.value


def _batch_ptrs(items):
    bs = [bytes(x) for x in items]
    k = len(bs)
    ptrs = (ctypes.c_void_p * k)(*[ctypes.cast(ctypes.c_char_p(x), ctypes.c_void_p).value for x in bs])
    lens = (ctypes.c_size_t * k)(*[len(x) for x in bs])
    return bs, ptrs, lens


def _batch_take(k, outs, olens):
    res = []
    for i in range(k):
        res.append(ctypes.string_at(outs[i], olens[i]) if outs[i] else b"")
        if outs[i]:
            lib.zt_free(outs[i])
    return res


def gzip_compress_batch(items, name=None, comment=None, hcrc=False, mtime=0, compression_type=2, lazy=0, level=-1):
    """GZip members of many buffers in one pipeline per device (config C4)."""
    bs, ptrs, lens = _batch_ptrs(items)
    k = len(bs)
    o = GzipOpts()
    o.deflate = DeflateOpts(compression_type, lazy, level)
    o.fname, o.fcomment, o.fhcrc, o.mtime = int(name is not None), int(comment is not None), int(hcrc), mtime
    if name is not None:
        o.name, o.name_len = bytes(name), len(name)
    if comment is not None:
        o.comment, o.comment_len = bytes(comment), len(comment)
    outs = (ctypes.POINTER(ctypes.c_uint8) * k)()
    olens = (ctypes.c_size_t * k)()
    st = (ctypes.c_int * k)()
    _check(lib.zt_gzip_compress_batch(ptrs, lens, k, ctypes.byref(o), outs, olens, st))
    return _batch_take(k, outs, olens)


def zlib_compress_batch(items, compression_type=2, lazy=0, level=-1):
    bs, ptrs, lens = _batch_ptrs(items)
    k = len(bs)
    opts = DeflateOpts(compression_type, lazy, level)
    outs = (ctypes.POINTER(ctypes.c_uint8) * k)()
    olens = (ctypes.c_size_t * k)()
    st = (ctypes.c_int * k)()
    _check(lib.zt_zlib_compress_batch(ptrs, lens, k, ctypes.byref(opts), outs, olens, st))
    return _batch_take(k, outs, olens)


def crc32_batch(items):
    bs, ptrs, lens = _batch_ptrs(items)
    out = (ctypes.c_uint32 * len(bs))()
    _check(lib.zt_crc32_batch(ptrs, lens, len(bs), out))
    return list(out)


def dos_mtime(year, month, day, hour, minute, second):
    """The 4 DOS time / date bytes of src/Zip.ts:130-139 (month 1-12)."""
    return bytes([((minute & 7) << 5) | (second >> 1), ((hour << 3) | (minute >> 3)) & 0xFF,
                  ((month & 7) << 5) | day, (((year - 1980) & 0x7F) << 1) | (month >> 3)])


def zip_compress(files, comment=b""):
    """Zip.addFile(...) for each dict of `files` (data, name, comment, method,
    os, mtime = 4 DOS bytes, compression_type, lazy) then Zip.compress()."""
    k = len(files)
    datas = [bytes(f["data"]) for f in files]
    bs, ptrs, lens = _batch_ptrs(datas)
    arr = (ZipFile * k)()
    keep = []
    for i, f in enumerate(files):
        nm, cm = bytes(f.get("name", b"")), f.get("comment")
        keep += [nm, cm]
        arr[i].name, arr[i].name_len = nm, len(nm)
        if cm is not None:
            arr[i].comment, arr[i].comment_len = bytes(cm), len(cm)
        arr[i].method = f.get("method", 8)
        arr[i].os = f.get("os", 0)
        arr[i].mtime = (ctypes.c_uint8 * 4)(*f.get("mtime", b"\0\0\0\0"))
        arr[i].deflate = DeflateOpts(f.get("compression_type", 2), f.get("lazy", 0), f.get("level", -1))
    out = ctypes.POINTER(ctypes.c_uint8)()
    olen = ctypes.c_size_t()
    cb = bytes(comment)
    _check(lib.zt_zip_compress(ptrs, lens, arr, k, cb, len(cb), ctypes.byref(out), ctypes.byref(olen)))
    return _take(out, olen)


def unzip(archive, verify=False):
    """Unzip every entry.  Returns (first error or None, [entry dicts with
    name, comment, data (or None), status, message and the header fields])."""
    b, n = _cbuf(archive)
    archive = bytes(archive)
    out = ctypes.POINTER(ctypes.c_uint8)()
    olen = ctypes.c_size_t()
    ents = ctypes.POINTER(UnzipEntry)()
    cnt = ctypes.c_size_t()
    rc = lib.zt_unzip(b, n, int(verify), ctypes.byref(out), ctypes.byref(olen), ctypes.byref(ents), ctypes.byref(cnt))
    if rc != ZT_OK and not ents:
        return ZtError(rc, lib.zt_last_error_message().decode(errors="replace")), []
    data = ctypes.string_at(out, olen.value) if out else b""
    res = []
    for i in range(cnt.value):
        e = ents[i]
        d = {f: getattr(e, f) for f, _ in UnzipEntry._fields_ if f != "message"}
        d["message"] = e.message.decode(errors="replace")
        d["name"] = archive[e.name_off:e.name_off + e.name_len]
        d["comment"] = archive[e.comment_off:e.comment_off + e.comment_len]
        d["data"] = data[e.data_off:e.data_off + e.data_len] if e.status == 0 else None
        res.append(d)
    if out:
        lib.zt_free(out)
    if ents:
        lib.zt_free(ents)
    err = None if rc == ZT_OK else ZtError(rc, lib.zt_last_error_message().decode(errors="replace"))
    return err, res


def gunzip(data):
    """GUnzip.decompress + getMembers (src/GUnzip.ts:43-175).  Returns
    (output, [member dicts])."""
    b, n = _cbuf(data)
    raw = bytes(data)
    out = ctypes.POINTER(ctypes.c_uint8)()
    olen = ctypes.c_size_t()
    mem = ctypes.POINTER(GzipMember)()
    cnt = ctypes.c_size_t()
    _check(lib.zt_gunzip(b, n, ctypes.byref(out), ctypes.byref(olen), ctypes.byref(mem), ctypes.byref(cnt)))
    res = _take(out, olen)
    members = []
    for i in range(cnt.value):
        m = mem[i]
        d = {k: getattr(m, k) for k, _ in GzipMember._fields_}
        d["name"] = raw[m.name_off:m.name_off + m.name_len] if m.flg & 0x08 else None
        d["comment"] = raw[m.comment_off:m.comment_off + m.comment_len] if m.flg & 0x10 else None
        d["data"] = res[m.data_off:m.data_off + m.data_len]
        members.append(d)
    lib.zt_free(mem)
    return res, members


def zlib_compress(data, compression_type=2, lazy=0, level=-1):
    """Deflate.compress (src/Deflate.ts:60-99).  Returns (stream, adler32)."""
    b, n = _cbuf(data)
    o = DeflateOpts(compression_type, lazy, level)
    out = ctypes.POINTER(ctypes.c_uint8)()
    olen = ctypes.c_size_t()
    adler = ctypes.c_uint32()
    _check(lib.zt_zlib_compress(b, n, ctypes.byref(o), ctypes.byref(out), ctypes.byref(olen), ctypes.byref(adler)))
    return _take(out, olen), adler.value


def zlib_decompress(data, index=0, verify=False):
    """Inflate.decompress (src/Inflate.ts:34-93).  Returns (output, ip)."""
    b, n = _cbuf(data)
    out = ctypes.POINTER(ctypes.c_uint8)()
    olen = ctypes.c_size_t()
    ip = ctypes.c_size_t()
    adler = ctypes.c_uint32()
    _check(lib.zt_zlib_decompress(b, n, index, int(verify), ctypes.byref(out), ctypes.byref(olen), ctypes.byref(ip),
                                  ctypes.byref(adler)))
    return _take(out, olen), ip.value


# ---- device-resident helpers (torch tensors as HBM buffers) -----------------------
def dev_checksums(ptr, n, crc=0, adler=1, stream=None):
    c, a = ctypes.c_uint32(), ctypes.c_uint32()
    _check(lib.zt_dev_checksums(ptr, n, crc, adler, ctypes.byref(c), ctypes.byref(a), stream))
    return c.value, a.value


class DeflatePlan:
    def __init__(self, max_n, level=-1, compression_type=2):
        self.h = ctypes.c_void_p()
        opts = DeflateOpts(compression_type, 0, level)
        _check(lib.zt_deflate_plan_create(max_n, ctypes.byref(opts), ctypes.byref(self.h)))

    def run(self, d_in, n, d_out, halo=0, final=1, stream=None):
        olen = ctypes.c_size_t()
        _check(lib.zt_deflate_dev(self.h, d_in, n, halo, final, d_out, ctypes.byref(olen), stream))
        return olen.value

    def close(self):
        if self.h and lib is not None:
            lib.zt_deflate_plan_destroy(self.h)
            self.h = ctypes.c_void_p()

    __del__ = close


class InflatePlan:
    def __init__(self, max_in, max_out):
        self.h = ctypes.c_void_p()
        _check(lib.zt_inflate_plan_create(max_in, max_out, ctypes.byref(self.h)))

    def run(self, d_in, n, d_out, out_cap, stream=None):
        olen, ip = ctypes.c_size_t(), ctypes.c_size_t()
        _check(lib.zt_inflate_dev(self.h, d_in, n, d_out, out_cap, ctypes.byref(olen), ctypes.byref(ip), stream))
        return olen.value, ip.value

    def close(self):
        if self.h and lib is not None:
            lib.zt_inflate_plan_destroy(self.h)
            self.h = ctypes.c_void_p()

    __del__ = close


def deflate_bound(n):
    return lib.zt_deflate_bound(n)


GEN_KINDS = {"xorshift32": 0, "wordsalad": 1, "structured": 2, "mixed": 3}


def synth_dev(kind, seed, ptr, n, stream=None):
    """Fill device memory with a synthetic corpus (64 KiB piece i = generator
    seeded with seed + i)."""
    _check(lib.zt_synth_dev(GEN_KINDS.get(kind, kind), seed, ptr, n, stream))


def synth_dev_at(kind, seed, offset, ptr, n, stream=None):
    """Bytes [offset, offset + n) of the corpus synth_dev would write from 0
    (offset a multiple of 64 KiB): one rank's shard of a sharded buffer."""
    if offset % 65536:
        raise ValueError("offset must be a multiple of 64 KiB")
    _check(lib.zt_synth_dev_at(GEN_KINDS.get(kind, kind), seed, offset // 65536, ptr, n, stream))


def timing_enable(on=True):
    _check(lib.zt_timing_enable(1 if on else 0))


def timing_read():
    t = KernelTimes()
    _check(lib.zt_timing_read(ctypes.byref(t)))
    return {"deflate_ms": t.deflate_ms, "deflate_launches": t.deflate_launches,
            "inflate_ms": t.inflate_ms, "inflate_launches": t.inflate_launches,
            "deflate_pipeline_ms": t.deflate_pipeline_ms, "deflate_pipelines": t.deflate_pipelines,
            "inflate_tok_ms": t.inflate_tok_ms, "inflate_toks": t.inflate_toks,
            "inflate_paths": list(t.inflate_paths), "general_passes": t.general_passes,
            "blocks_unsearched": t.blocks_unsearched}


def scratch_bytes():
    """(device scratch, pinned host staging) bytes the device context caches."""
    d, h = ctypes.c_size_t(0), ctypes.c_size_t(0)
    _check(lib.zt_scratch_bytes(ctypes.byref(d), ctypes.byref(h)))
    return d.value, h.value


def release_scratch():
    _check(lib.zt_release_scratch())
