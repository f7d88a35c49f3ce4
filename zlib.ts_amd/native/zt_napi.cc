// zt_napi.cc -- N-API addon: the thin binding between the JS facade
// (zlib.ts_amd/lib/*.js, the reference's RawDeflate / RawInflate / CRC32 /
// Adler32 surface) and libzt.so's C-ABI (include/zt.h).  Uint8Array memory is
// passed zero-copy; results come back as Uint8Arrays over the library's own
// output buffers (no copy, released by zt_free on collection).  Every call runs on
// the GPU; errors carry libzt's status code and message (the JS facade maps
// them onto the reference's thrown values).
#include <node_api.h>

#include <cstdio>
#include <cstring>
#include <vector>

#include "../../include/zt.h"

namespace {

napi_value throw_zt(napi_env env, int code) {
  const char *msg = zt_last_error_message();
  char codebuf[16];
  snprintf(codebuf, sizeof codebuf, "%d", code);
  napi_value err, m, c;
  napi_create_string_utf8(env, msg ? msg : "libzt error", NAPI_AUTO_LENGTH, &m);
  napi_create_string_utf8(env, codebuf, NAPI_AUTO_LENGTH, &c);
  napi_create_error(env, c, m, &err);
  napi_value num;
  napi_create_int32(env, code, &num);
  napi_set_named_property(env, err, "ztStatus", num);
  napi_throw(env, err);
  return nullptr;
}

bool get_u8(napi_env env, napi_value v, const uint8_t **p, size_t *n) {
  bool is_ta = false;
  napi_is_typedarray(env, v, &is_ta);
  if (!is_ta) {
    napi_throw_type_error(env, nullptr, "expected a Uint8Array");
    return false;
  }
  napi_typedarray_type t;
  size_t len = 0, off = 0;
  void *data = nullptr;
  napi_value ab;
  napi_get_typedarray_info(env, v, &t, &len, &data, &ab, &off);
  if (t != napi_uint8_array) {
    napi_throw_type_error(env, nullptr, "expected a Uint8Array");
    return false;
  }
  *p = static_cast<const uint8_t *>(data);
  *n = len;
  return true;
}

int64_t get_i64(napi_env env, napi_value v, int64_t dflt) {
  napi_valuetype t;
  napi_typeof(env, v, &t);
  if (t != napi_number) return dflt;
  int64_t x = dflt;
  napi_get_value_int64(env, v, &x);
  return x;
}

uint32_t get_u32(napi_env env, napi_value v, uint32_t dflt) {
  napi_valuetype t;
  napi_typeof(env, v, &t);
  if (t != napi_number) return dflt;
  uint32_t x = dflt;
  napi_get_value_uint32(env, v, &x);
  return x;
}

// A libzt-allocated result handed to JS without a copy: an external
// ArrayBuffer over the library's buffer, released by zt_free when the GC
// collects it (large outputs then go back to libzt's host output pool,
// registered for DMA, and the next call of a similar size reuses them).  The
// bytes are reported to V8 as external memory so that a loop of large calls
// triggers collections.
void release_result(napi_env env, void *data, void *hint) {
  zt_free(data);
  int64_t adj = 0;
  napi_adjust_external_memory(env, -(int64_t)(uintptr_t)hint, &adj);
}

napi_value new_u8(napi_env env, uint8_t *buf, size_t n) {
  napi_value ab, ta;
  if (n == 0 || !buf) {
    void *data = nullptr;
    napi_create_arraybuffer(env, 0, &data, &ab);
    zt_free(buf);
  } else if (napi_create_external_arraybuffer(env, buf, n, release_result, (void *)(uintptr_t)n, &ab) == napi_ok) {
    int64_t adj = 0;
    napi_adjust_external_memory(env, (int64_t)n, &adj);
  } else {  // (a runtime without external buffers: copy)
    void *data = nullptr;
    napi_create_arraybuffer(env, n, &data, &ab);
    memcpy(data, buf, n);
    zt_free(buf);
  }
  napi_create_typedarray(env, napi_uint8_array, n, ab, 0, &ta);
  return ta;
}

napi_value args(napi_env env, napi_callback_info info, napi_value *argv, size_t want) {
  size_t argc = want;
  napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr);
  napi_value undef;
  napi_get_undefined(env, &undef);
  for (size_t i = argc; i < want; ++i) argv[i] = undef;
  return undef;
}

// crc32Update(data: Uint8Array, crc: number) -> number
napi_value crc32_update(napi_env env, napi_callback_info info) {
  napi_value a[2];
  args(env, info, a, 2);
  const uint8_t *p;
  size_t n;
  if (!get_u8(env, a[0], &p, &n)) return nullptr;
  uint32_t out = 0;
  int rc = zt_crc32_update(get_u32(env, a[1], 0), p, n, &out);
  if (rc) return throw_zt(env, rc);
  napi_value r;
  napi_create_uint32(env, out, &r);
  return r;
}

// adler32Update(adler: number, data: Uint8Array) -> number
napi_value adler32_update(napi_env env, napi_callback_info info) {
  napi_value a[2];
  args(env, info, a, 2);
  const uint8_t *p;
  size_t n;
  if (!get_u8(env, a[1], &p, &n)) return nullptr;
  uint32_t out = 0;
  int rc = zt_adler32_update(get_u32(env, a[0], 1), p, n, &out);
  if (rc) return throw_zt(env, rc);
  napi_value r;
  napi_create_uint32(env, out, &r);
  return r;
}

// deflateRaw(input: Uint8Array, compressionType, lazy, level) -> Uint8Array
napi_value deflate_raw(napi_env env, napi_callback_info info) {
  napi_value a[4];
  args(env, info, a, 4);
  const uint8_t *p;
  size_t n;
  if (!get_u8(env, a[0], &p, &n)) return nullptr;
  zt_deflate_opts o;
  o.compression_type = (int)get_i64(env, a[1], 2);
  o.lazy = (int)get_i64(env, a[2], 0);
  o.level = (int)get_i64(env, a[3], -1);
  uint8_t *out = nullptr;
  size_t olen = 0;
  int rc = zt_deflate_raw(p, n, &o, &out, &olen);
  if (rc) return throw_zt(env, rc);
  return new_u8(env, out, olen);
}

// inflateRaw(input: Uint8Array, index, bufferType, bufferSize, refStrict) -> {output, ip}
napi_value inflate_raw(napi_env env, napi_callback_info info) {
  napi_value a[5];
  args(env, info, a, 5);
  const uint8_t *p;
  size_t n;
  if (!get_u8(env, a[0], &p, &n)) return nullptr;
  const int64_t index = get_i64(env, a[1], 0);
  zt_inflate_opts o;
  o.buffer_type = (int)get_i64(env, a[2], 1);
  o.buffer_size = (size_t)get_i64(env, a[3], 0x8000);
  bool strict = false;
  napi_valuetype t;
  napi_typeof(env, a[4], &t);
  if (t == napi_boolean) napi_get_value_bool(env, a[4], &strict);
  o.ref_strict = strict ? 1 : 0;
  uint8_t *out = nullptr;
  size_t olen = 0, ip = 0;
  int rc = zt_inflate_raw(p, n, index < 0 ? 0 : (size_t)index, &o, &out, &olen, &ip);
  if (rc) return throw_zt(env, rc);
  napi_value obj, ipv;
  napi_create_object(env, &obj);
  napi_set_named_property(env, obj, "output", new_u8(env, out, olen));
  napi_create_double(env, (double)ip, &ipv);
  napi_set_named_property(env, obj, "ip", ipv);
  return obj;
}

void set_num(napi_env env, napi_value obj, const char *k, double v) {
  napi_value x;
  napi_create_double(env, v, &x);
  napi_set_named_property(env, obj, k, x);
}

// inflateResume(input: Uint8Array, bitPos, window: Uint8Array[, final]) -> {output, endBits, finished}
// (final: no more input will come -- zt_inflate_raw_resume_final)
napi_value inflate_resume(napi_env env, napi_callback_info info) {
  napi_value a[4];
  args(env, info, a, 4);
  const uint8_t *p, *w;
  size_t n, wn;
  if (!get_u8(env, a[0], &p, &n) || !get_u8(env, a[2], &w, &wn)) return nullptr;
  const int64_t bit = get_i64(env, a[1], 0);
  uint8_t *out = nullptr;
  size_t olen = 0;
  uint64_t end = 0;
  int fin = 0;
  const bool final_input = get_i64(env, a[3], 0) != 0;
  int rc = (final_input ? zt_inflate_raw_resume_final : zt_inflate_raw_resume)(p, n, bit < 0 ? 0 : (uint64_t)bit, w,
                                                                               wn, &out, &olen, &end, &fin);
  if (rc) return throw_zt(env, rc);
  napi_value obj, f;
  napi_create_object(env, &obj);
  napi_set_named_property(env, obj, "output", new_u8(env, out, olen));
  set_num(env, obj, "endBits", (double)end);
  napi_get_boolean(env, fin != 0, &f);
  napi_set_named_property(env, obj, "finished", f);
  return obj;
}

// optional Uint8Array argument (undefined / null -> absent)
bool opt_u8(napi_env env, napi_value v, const uint8_t **p, size_t *n, bool *present) {
  napi_valuetype t;
  napi_typeof(env, v, &t);
  *present = !(t == napi_undefined || t == napi_null);
  *p = nullptr;
  *n = 0;
  return !*present || get_u8(env, v, p, n);
}

// gzipCompress(input, compressionType, lazy, level, name|null, comment|null, hcrc, mtime) -> {output, crc32}
napi_value gzip_compress(napi_env env, napi_callback_info info) {
  napi_value a[8];
  args(env, info, a, 8);
  const uint8_t *p;
  size_t n;
  if (!get_u8(env, a[0], &p, &n)) return nullptr;
  zt_gzip_opts o;
  memset(&o, 0, sizeof o);
  o.deflate.compression_type = (int)get_i64(env, a[1], 2);
  o.deflate.lazy = (int)get_i64(env, a[2], 0);
  o.deflate.level = (int)get_i64(env, a[3], -1);
  bool has = false;
  if (!opt_u8(env, a[4], &o.name, &o.name_len, &has)) return nullptr;
  o.fname = has;
  if (!opt_u8(env, a[5], &o.comment, &o.comment_len, &has)) return nullptr;
  o.fcomment = has;
  bool hcrc = false;
  napi_valuetype t;
  napi_typeof(env, a[6], &t);
  if (t == napi_boolean) napi_get_value_bool(env, a[6], &hcrc);
  o.fhcrc = hcrc;
  o.mtime = get_u32(env, a[7], 0);
  uint8_t *out = nullptr;
  size_t olen = 0;
  uint32_t crc = 0;
  int rc = zt_gzip_compress(p, n, &o, &out, &olen, &crc);
  if (rc) return throw_zt(env, rc);
  napi_value obj;
  napi_create_object(env, &obj);
  napi_set_named_property(env, obj, "output", new_u8(env, out, olen));
  set_num(env, obj, "crc32", crc);
  return obj;
}

// gunzip(input) -> {output, members: [{flg, mtime, xfl, os, xlen, nameOff, nameLen, commentOff,
//                   commentLen, crc16 (or -1), crc32, isize, dataOff, dataLen}]}
napi_value gunzip(napi_env env, napi_callback_info info) {
  napi_value a[1];
  args(env, info, a, 1);
  const uint8_t *p;
  size_t n;
  if (!get_u8(env, a[0], &p, &n)) return nullptr;
  uint8_t *out = nullptr;
  size_t olen = 0, cnt = 0;
  zt_gzip_member *mem = nullptr;
  int rc = zt_gunzip(p, n, &out, &olen, &mem, &cnt);
  if (rc) return throw_zt(env, rc);
  napi_value obj, arr;
  napi_create_object(env, &obj);
  napi_set_named_property(env, obj, "output", new_u8(env, out, olen));
  napi_create_array_with_length(env, cnt, &arr);
  for (size_t i = 0; i < cnt; ++i) {
    const zt_gzip_member &m = mem[i];
    napi_value e;
    napi_create_object(env, &e);
    set_num(env, e, "flg", m.flg);
    set_num(env, e, "mtime", m.mtime);
    set_num(env, e, "xfl", m.xfl);
    set_num(env, e, "os", m.os);
    set_num(env, e, "xlen", m.xlen);
    set_num(env, e, "nameOff", (double)m.name_off);
    set_num(env, e, "nameLen", (double)m.name_len);
    set_num(env, e, "commentOff", (double)m.comment_off);
    set_num(env, e, "commentLen", (double)m.comment_len);
    set_num(env, e, "crc16", m.has_crc16 ? (double)m.crc16 : -1.0);
    set_num(env, e, "crc32", m.crc32);
    set_num(env, e, "isize", m.isize);
    set_num(env, e, "dataOff", (double)m.data_off);
    set_num(env, e, "dataLen", (double)m.data_len);
    napi_set_element(env, arr, (uint32_t)i, e);
  }
  zt_free(mem);
  napi_set_named_property(env, obj, "members", arr);
  return obj;
}

// zlibCompress(input, compressionType, lazy, level) -> {output, adler32}
napi_value zlib_compress(napi_env env, napi_callback_info info) {
  napi_value a[4];
  args(env, info, a, 4);
  const uint8_t *p;
  size_t n;
  if (!get_u8(env, a[0], &p, &n)) return nullptr;
  zt_deflate_opts o;
  o.compression_type = (int)get_i64(env, a[1], 2);
  o.lazy = (int)get_i64(env, a[2], 0);
  o.level = (int)get_i64(env, a[3], -1);
  uint8_t *out = nullptr;
  size_t olen = 0;
  uint32_t adler = 1;
  int rc = zt_zlib_compress(p, n, &o, &out, &olen, &adler);
  if (rc) return throw_zt(env, rc);
  napi_value obj;
  napi_create_object(env, &obj);
  napi_set_named_property(env, obj, "output", new_u8(env, out, olen));
  set_num(env, obj, "adler32", adler);
  return obj;
}

// zlibDecompress(input, index, verify) -> {output, ip, adler32}
napi_value zlib_decompress(napi_env env, napi_callback_info info) {
  napi_value a[3];
  args(env, info, a, 3);
  const uint8_t *p;
  size_t n;
  if (!get_u8(env, a[0], &p, &n)) return nullptr;
  const int64_t index = get_i64(env, a[1], 0);
  bool verify = false;
  napi_valuetype t;
  napi_typeof(env, a[2], &t);
  if (t == napi_boolean) napi_get_value_bool(env, a[2], &verify);
  uint8_t *out = nullptr;
  size_t olen = 0, ip = 0;
  uint32_t adler = 1;
  int rc = zt_zlib_decompress(p, n, index < 0 ? 0 : (size_t)index, verify, &out, &olen, &ip, &adler);
  if (rc) return throw_zt(env, rc);
  napi_value obj;
  napi_create_object(env, &obj);
  napi_set_named_property(env, obj, "output", new_u8(env, out, olen));
  set_num(env, obj, "ip", (double)ip);
  set_num(env, obj, "adler32", adler);
  return obj;
}

napi_value prop(napi_env env, napi_value obj, const char *k) {
  napi_value v;
  napi_get_named_property(env, obj, k, &v);
  return v;
}

// zipCompress(files: [{data, name, comment (or null), method, os, mtime (4 bytes),
//             compressionType, lazy, level}], comment: Uint8Array) -> Uint8Array
napi_value zip_compress(napi_env env, napi_callback_info info) {
  napi_value a[2];
  args(env, info, a, 2);
  uint32_t cnt = 0;
  napi_get_array_length(env, a[0], &cnt);
  std::vector<const uint8_t *> in(cnt);
  std::vector<size_t> n(cnt);
  std::vector<zt_zip_file> f(cnt);
  for (uint32_t i = 0; i < cnt; ++i) {
    napi_value e;
    napi_get_element(env, a[0], i, &e);
    memset(&f[i], 0, sizeof f[i]);
    if (!get_u8(env, prop(env, e, "data"), &in[i], &n[i])) return nullptr;
    if (!get_u8(env, prop(env, e, "name"), &f[i].name, &f[i].name_len)) return nullptr;
    bool has = false;
    if (!opt_u8(env, prop(env, e, "comment"), &f[i].comment, &f[i].comment_len, &has)) return nullptr;
    f[i].method = (int)get_i64(env, prop(env, e, "method"), 8);
    f[i].os = (int)get_i64(env, prop(env, e, "os"), 0);
    const uint8_t *mt;
    size_t ml;
    if (!get_u8(env, prop(env, e, "mtime"), &mt, &ml)) return nullptr;
    for (size_t k = 0; k < 4 && k < ml; ++k) f[i].mtime[k] = mt[k];
    f[i].deflate.compression_type = (int)get_i64(env, prop(env, e, "compressionType"), 2);
    f[i].deflate.lazy = (int)get_i64(env, prop(env, e, "lazy"), 0);
    f[i].deflate.level = (int)get_i64(env, prop(env, e, "level"), -1);
  }
  const uint8_t *cm = nullptr;
  size_t cl = 0;
  bool has = false;
  if (!opt_u8(env, a[1], &cm, &cl, &has)) return nullptr;
  uint8_t *out = nullptr;
  size_t olen = 0;
  const int rc = zt_zip_compress(in.data(), n.data(), f.data(), cnt, cm, cl, &out, &olen);
  if (rc) return throw_zt(env, rc);
  return new_u8(env, out, olen);
}

// unzip(input, verify) -> {output, entries: [{nameOff, nameLen, ..., status, message}]}
// (archive-level errors throw; an entry's error is in its status / message)
napi_value unzip(napi_env env, napi_callback_info info) {
  napi_value a[2];
  args(env, info, a, 2);
  const uint8_t *p;
  size_t n;
  if (!get_u8(env, a[0], &p, &n)) return nullptr;
  bool verify = false;
  napi_valuetype t;
  napi_typeof(env, a[1], &t);
  if (t == napi_boolean) napi_get_value_bool(env, a[1], &verify);
  uint8_t *out = nullptr;
  size_t olen = 0, cnt = 0;
  zt_unzip_entry *ent = nullptr;
  const int rc = zt_unzip(p, n, verify ? 1 : 0, &out, &olen, &ent, &cnt);
  if (rc && !ent) return throw_zt(env, rc);
  napi_value obj, arr;
  napi_create_object(env, &obj);
  napi_set_named_property(env, obj, "output", new_u8(env, out, olen));
  napi_create_array_with_length(env, cnt, &arr);
  for (size_t i = 0; i < cnt; ++i) {
    const zt_unzip_entry &m = ent[i];
    napi_value e;
    napi_create_object(env, &e);
    set_num(env, e, "nameOff", (double)m.name_off);
    set_num(env, e, "nameLen", (double)m.name_len);
    set_num(env, e, "commentOff", (double)m.comment_off);
    set_num(env, e, "commentLen", (double)m.comment_len);
    set_num(env, e, "dataOff", (double)m.data_off);
    set_num(env, e, "dataLen", (double)m.data_len);
    set_num(env, e, "relativeOffset", (double)m.local_offset);
    set_num(env, e, "version", m.version);
    set_num(env, e, "os", m.os);
    set_num(env, e, "needVersion", m.need_version);
    set_num(env, e, "flags", m.flags);
    set_num(env, e, "compression", m.method);
    set_num(env, e, "time", m.time);
    set_num(env, e, "date", m.date);
    set_num(env, e, "crc32", m.crc32);
    set_num(env, e, "compressedSize", m.compressed_size);
    set_num(env, e, "plainSize", m.plain_size);
    set_num(env, e, "status", m.status);
    napi_value msg;
    napi_create_string_utf8(env, m.message, NAPI_AUTO_LENGTH, &msg);
    napi_set_named_property(env, e, "message", msg);
    napi_set_element(env, arr, (uint32_t)i, e);
  }
  zt_free(ent);
  napi_set_named_property(env, obj, "entries", arr);
  return obj;
}

napi_value device_count(napi_env env, napi_callback_info) {
  napi_value r;
  napi_create_int32(env, zt_device_count(), &r);
  return r;
}

napi_value version(napi_env env, napi_callback_info) {
  napi_value r;
  napi_create_string_utf8(env, zt_version(), NAPI_AUTO_LENGTH, &r);
  return r;
}

napi_value init(napi_env env, napi_value exports) {
  napi_property_descriptor d[] = {
      {"crc32Update", nullptr, crc32_update, nullptr, nullptr, nullptr, napi_enumerable, nullptr},
      {"adler32Update", nullptr, adler32_update, nullptr, nullptr, nullptr, napi_enumerable, nullptr},
      {"deflateRaw", nullptr, deflate_raw, nullptr, nullptr, nullptr, napi_enumerable, nullptr},
      {"inflateRaw", nullptr, inflate_raw, nullptr, nullptr, nullptr, napi_enumerable, nullptr},
      {"inflateResume", nullptr, inflate_resume, nullptr, nullptr, nullptr, napi_enumerable, nullptr},
      {"gzipCompress", nullptr, gzip_compress, nullptr, nullptr, nullptr, napi_enumerable, nullptr},
      {"gunzip", nullptr, gunzip, nullptr, nullptr, nullptr, napi_enumerable, nullptr},
      {"zlibCompress", nullptr, zlib_compress, nullptr, nullptr, nullptr, napi_enumerable, nullptr},
      {"zlibDecompress", nullptr, zlib_decompress, nullptr, nullptr, nullptr, napi_enumerable, nullptr},
      {"zipCompress", nullptr, zip_compress, nullptr, nullptr, nullptr, napi_enumerable, nullptr},
      {"unzip", nullptr, unzip, nullptr, nullptr, nullptr, napi_enumerable, nullptr},
      {"deviceCount", nullptr, device_count, nullptr, nullptr, nullptr, napi_enumerable, nullptr},
      {"version", nullptr, version, nullptr, nullptr, nullptr, napi_enumerable, nullptr},
  };
  napi_define_properties(env, exports, sizeof d / sizeof d[0], d);
  return exports;
}

}  // namespace

NAPI_MODULE(NODE_GYP_MODULE_NAME, init)
