// container_api.cpp -- GZip (RFC 1952) and zlib (RFC 1950) containers over the
// raw DEFLATE engine (include/zt.h).
//
// Headers and trailers are a few bytes of host logic; the hot path stays on
// the GPU: GZip compress uploads the input once and runs the deflate pipeline
// and the CRC-32 kernel on the same device-resident bytes (the reference
// deflates and then walks the input a second time for the CRC,
// src/GZip.ts:164-180); zlib compress does the same with Adler-32.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "zt_internal.h"

namespace zt {

size_t deflate_bound_bytes(size_t n);
size_t deflate_scratch_bytes(const DeviceCtx *c, size_t n);
int deflate_dev_run(DeviceCtx *c, const uint8_t *d_in, size_t n, size_t halo, int final_, int ctype, int level,
                    uint8_t *d_out, size_t *out_len, void *scratch_base, size_t scratch_size, hipStream_t s);

namespace {

int resolve_deflate(const zt_deflate_opts *o, int *ctype, int *level) {
  int ct = o ? o->compression_type : 2;
  int lv = o ? o->level : -1;
  if (ct < 0 || ct > 2) return set_error(ZT_E_INVALID_COMPRESSION_TYPE, "invalid compression type");
  if (lv < 0 || lv > 9) lv = 6;
  if (lv == 0) ct = 0;
  if (o && o->lazy > 0 && lv < 4) lv = 4;
  *ctype = ct;
  *level = lv;
  return ZT_OK;
}

// Raw DEFLATE of host bytes into `out` after `prefix` bytes of header, with the
// input's CRC-32 and/or Adler-32 from the same device copy of the input.
// *out (malloc'd) = prefix | stream | `trailer` bytes of room.
int deflate_with_checksums(const uint8_t *in, size_t n, const zt_deflate_opts *opts, const uint8_t *prefix,
                           size_t prefix_len, size_t trailer, uint8_t **out, size_t *stream_len, uint32_t *crc,
                           uint32_t *adler) {
  DeviceCtx *c;
  ZT_TRY(get_ctx(&c));
  std::lock_guard<std::recursive_mutex> ctx_lock(c->mu);
  int ct, lv;
  ZT_TRY(resolve_deflate(opts, &ct, &lv));
  const size_t ob = (ct == 0 ? n + 5 * ((n + 65534) / 65535) + 16 : deflate_bound_bytes(n) + (ct == 1 ? n / 8 + 64 : 0));
  void *d_in, *d_out, *d_scr, *d_res;
  ZT_TRY(scratch(c, 0, n + 64, &d_in));
  ZT_TRY(scratch(c, 1, ob, &d_out));
  const size_t ss = deflate_scratch_bytes(c, n);
  ZT_TRY(scratch(c, 3, ss, &d_scr));
  ZT_TRY(scratch(c, 2, 16, &d_res));
  ZT_TRY(upload(c, d_in, in, n, c->stream));
  // the checksums run on the second stream beside the deflate pipeline (both
  // only read the input); every return below waits for that stream first
  uint32_t sums[2] = {0, 1};  // CRC-32 and Adler-32 of nothing
  struct AuxWait {
    hipStream_t s;
    ~AuxWait() { (void)hipStreamSynchronize(s); }
  } aux_wait{c->aux};
  if (n) {
    ZT_HIP(hipEventRecord(c->aux_ev, c->stream));
    ZT_HIP(hipStreamWaitEvent(c->aux, c->aux_ev, 0));
    ZT_TRY(checksums_dev(c, (const uint8_t *)d_in, n, crc != nullptr, adler != nullptr, 0, 1, (uint32_t *)d_res,
                         c->aux));
    ZT_HIP(hipMemcpyAsync(sums, d_res, sizeof sums, hipMemcpyDeviceToHost, c->aux));
  }
  size_t len = 0;
  ZT_TRY(deflate_dev_run(c, (const uint8_t *)d_in, n, 0, 1, ct, lv, (uint8_t *)d_out, &len, d_scr, ss, c->stream));
  uint8_t *h = host_out(prefix_len + len + trailer + 1);
  if (!h) return set_error(ZT_E_NOMEM, "host allocation failed");
  if (prefix_len) memcpy(h, prefix, prefix_len);
  if (const int rc = download(c, h + prefix_len, d_out, len, c->stream)) {
    zt_free(h);
    return rc;
  }
  hipError_t e = hipStreamSynchronize(c->aux);
  if (e != hipSuccess) {
    zt_free(h);
    return hip_fail(e, "hipStreamSynchronize");
  }
  if (crc) *crc = sums[0];
  if (adler) *adler = sums[1];
  *out = h;
  *stream_len = len;
  return ZT_OK;
}

void put32le(uint8_t *p, uint32_t v) {
  p[0] = v & 0xFF;
  p[1] = (v >> 8) & 0xFF;
  p[2] = (v >> 16) & 0xFF;
  p[3] = v >> 24;
}

// CRC-32 of a few host bytes (headers): table-free bitwise form, host logic only
uint32_t crc32_small(const uint8_t *p, size_t n) {
  uint32_t c = 0xFFFFFFFFu;
  for (size_t i = 0; i < n; ++i) {
    c ^= p[i];
    for (int k = 0; k < 8; ++k) c = (c >> 1) ^ (0xEDB88320u & (0u - (c & 1u)));
  }
  return ~c;
}

// A byte of the input, or -1 past its end (the reference reads `undefined`).
// u8(): the value a JS bitwise expression gives that byte (`undefined | x`
// counts it as 0: ByteStream.readUint/readShort/readUintBE, src/ByteStream.ts:52-83).
struct Reader {
  const uint8_t *in;
  size_t n, p;
  int byte() { return p < n ? in[p++] : (++p, -1); }
  uint32_t u8() { return p < n ? in[p++] : (++p, 0u); }
};

std::string num(int v) { return v < 0 ? std::string("undefined") : std::to_string(v); }

}  // namespace

// member header: src/GZip.ts:104-158
void gzip_header(const zt_gzip_opts *opts, std::vector<uint8_t> &hd) {
  hd = {0x1F, 0x8B, 8};
  uint8_t flg = 0;
  if (opts && opts->fname) flg |= 0x08;
  if (opts && opts->fcomment) flg |= 0x10;
  if (opts && opts->fhcrc) flg |= 0x02;
  hd.push_back(flg);
  const uint32_t mtime = opts ? opts->mtime : 0;
  for (int k = 0; k < 4; ++k) hd.push_back((mtime >> (8 * k)) & 0xFF);
  hd.push_back(0);  // XFL
  hd.push_back(3);  // OS: UNIX (src/GZip.ts:128)
  if (opts && opts->fname) {
    hd.insert(hd.end(), opts->name, opts->name + opts->name_len);
    hd.push_back(0);
  }
  if (opts && opts->fcomment) {
    hd.insert(hd.end(), opts->comment, opts->comment + opts->comment_len);
    hd.push_back(0);
  }
  if (opts && opts->fhcrc) {
    const uint32_t c16 = crc32_small(hd.data(), hd.size()) & 0xFFFF;
    hd.push_back(c16 & 0xFF);
    hd.push_back(c16 >> 8);
  }
}
}  // namespace zt

using namespace zt;

extern "C" {

int zt_gzip_compress(const uint8_t *in, size_t n, const zt_gzip_opts *opts, uint8_t **out, size_t *out_len,
                     uint32_t *crc_out) {
  if (!out || !out_len) return set_error(ZT_E_ARG, "null output");
  if (n && !in) return set_error(ZT_E_ARG, "null input");
  std::vector<uint8_t> hd;
  gzip_header(opts, hd);
  uint8_t *buf;
  size_t slen;
  uint32_t crc;
  ZT_TRY(deflate_with_checksums(in, n, opts ? &opts->deflate : nullptr, hd.data(), hd.size(), 8, &buf, &slen, &crc,
                                nullptr));
  // trailer: CRC-32 and ISIZE (src/GZip.ts:179-185)
  put32le(buf + hd.size() + slen, crc);
  put32le(buf + hd.size() + slen + 4, (uint32_t)n);
  *out = buf;
  *out_len = hd.size() + slen + 8;
  if (crc_out) *crc_out = crc;
  return ZT_OK;
}

int zt_gunzip(const uint8_t *in, size_t n, uint8_t **out, size_t *out_len, zt_gzip_member **members,
              size_t *nmembers) {
  if (!out || !out_len) return set_error(ZT_E_ARG, "null output");
  if (n && !in) return set_error(ZT_E_ARG, "null input");
  std::vector<zt_gzip_member> mem;
  std::vector<uint8_t> data;
  size_t ip = 0;
  char msg[128];
  // the input goes to the device once; every member decodes from there
  DeviceCtx *c;
  ZT_TRY(get_ctx(&c));
  std::lock_guard<std::recursive_mutex> ctx_lock(c->mu);
  void *d_in = nullptr;
  if (n) {
    ZT_TRY(scratch(c, 19, n + 64, &d_in));
    ZT_TRY(upload(c, d_in, in, n, c->stream));
  }
  // src/GUnzip.ts:57-65: members until the input is consumed
  while (ip < n) {
    zt_gzip_member m;
    memset(&m, 0, sizeof m);
    Reader b{in, n, ip};
    const int id1 = b.byte(), id2 = b.byte();
    if (id1 != 0x1F || id2 != 0x8B) {
      snprintf(msg, sizeof msg, "invalid file signature:%s,%s", num(id1).c_str(), num(id2).c_str());
      return set_error(ZT_E_GZIP_SIGNATURE, msg);
    }
    const int cm = b.byte();
    if (cm != 8) {
      snprintf(msg, sizeof msg, "unknown compression method: %s", num(cm).c_str());
      return set_error(ZT_E_GZIP_METHOD, msg);
    }
    const int flg = b.byte();
    m.flg = (uint32_t)(flg < 0 ? 0 : flg);
    uint32_t mt = 0;
    for (int k = 0; k < 4; ++k) mt |= b.u8() << (8 * k);
    m.mtime = mt;
    m.xfl = b.u8();
    m.os = b.u8();
    if (m.flg & 0x04) {  // FEXTRA: skipped (src/GUnzip.ts:100-103,185-187)
      const uint32_t lo = b.u8(), hi = b.u8();
      m.xlen = lo | (hi << 8);
      b.p += m.xlen;
    }
    if (m.flg & 0x08) {  // FNAME
      m.name_off = b.p;
      int ch;
      while ((ch = b.byte()) > 0) {
      }
      m.name_len = b.p - 1 - m.name_off;
    }
    if (m.flg & 0x10) {  // FCOMMENT
      m.comment_off = b.p;
      int ch;
      while ((ch = b.byte()) > 0) {
      }
      m.comment_len = b.p - 1 - m.comment_off;
    }
    if (m.flg & 0x02) {
      // FHCRC: the reference takes the CRC of input[0 .. p), from the start of
      // the whole input, not of the member (src/GUnzip.ts:127-131)
      const uint32_t c16 = crc32_small(in, b.p < n ? b.p : n) & 0xFFFF;
      const uint32_t lo = b.u8(), hi = b.u8();
      m.has_crc16 = 1;
      m.crc16 = c16;
      if (c16 != (lo | (hi << 8))) return set_error(ZT_E_GZIP_HCRC, "invalid header crc16");
    }
    if (b.p > n) return set_error(ZT_E_INPUT_BROKEN, "input buffer is broken");
    // body (src/GUnzip.ts:149-153): the engine's RawInflate from index b.p
    uint8_t *o = nullptr;
    size_t olen = 0, eip = 0;
    ZT_TRY(inflate_dev_member(c, (const uint8_t *)d_in, n, b.p, &o, &olen, &eip));
    uint32_t crc = 0;
    const int rc = zt_crc32_update(0, o, olen, &crc);
    if (rc) {
      zt_free(o);
      return rc;
    }
    Reader t{in, n, eip};
    uint32_t want = 0, isize = 0;
    for (int k = 0; k < 4; ++k) want |= t.u8() << (8 * k);
    if (crc != want) {
      zt_free(o);
      snprintf(msg, sizeof msg, "invalid CRC-32 checksum: 0x%x / 0x%x", crc, want);
      return set_error(ZT_E_GZIP_CRC32, msg);
    }
    for (int k = 0; k < 4; ++k) isize |= t.u8() << (8 * k);
    if ((uint32_t)olen != isize) {
      zt_free(o);
      snprintf(msg, sizeof msg, "invalid input size: %u / %u", (uint32_t)olen, isize);
      return set_error(ZT_E_GZIP_ISIZE, msg);
    }
    m.crc32 = crc;
    m.isize = isize;
    m.data_off = data.size();
    m.data_len = olen;
    data.insert(data.end(), o, o + olen);
    zt_free(o);
    mem.push_back(m);
    ip = t.p;
  }
  uint8_t *h = host_out(data.size());
  if (!h) return set_error(ZT_E_NOMEM, "host allocation failed");
  if (!data.empty()) memcpy(h, data.data(), data.size());
  *out = h;
  *out_len = data.size();
  if (members) {
    *members = (zt_gzip_member *)malloc((mem.size() ? mem.size() : 1) * sizeof(zt_gzip_member));
    if (!*members) {
      zt_free(h);
      return set_error(ZT_E_NOMEM, "host allocation failed");
    }
    if (!mem.empty()) memcpy(*members, mem.data(), mem.size() * sizeof(zt_gzip_member));
  }
  if (nmembers) *nmembers = mem.size();
  return ZT_OK;
}

int zt_zlib_compress(const uint8_t *in, size_t n, const zt_deflate_opts *opts, uint8_t **out, size_t *out_len,
                     uint32_t *adler_out) {
  if (!out || !out_len) return set_error(ZT_E_ARG, "null output");
  if (n && !in) return set_error(ZT_E_ARG, "null input");
  const int ct = opts ? opts->compression_type : 2;
  if (ct < 0 || ct > 2) return set_error(ZT_E_INVALID_COMPRESSION_TYPE, "invalid compression type");
  // CMF = 0x78 (deflate, 32 KiB window); FLG: FLEVEL = compressionType, FCHECK (src/Deflate.ts:61-78)
  const uint32_t cmf = 0x78, flg0 = (uint32_t)ct << 6;
  const uint8_t hd[2] = {(uint8_t)cmf, (uint8_t)(flg0 | (31 - ((cmf << 8) + flg0) % 31))};
  uint8_t *buf;
  size_t slen;
  uint32_t adler;
  ZT_TRY(deflate_with_checksums(in, n, opts, hd, 2, 4, &buf, &slen, nullptr, &adler));
  // Adler-32, big-endian (src/Deflate.ts:95)
  uint8_t *t = buf + 2 + slen;
  t[0] = adler >> 24;
  t[1] = (adler >> 16) & 0xFF;
  t[2] = (adler >> 8) & 0xFF;
  t[3] = adler & 0xFF;
  *out = buf;
  *out_len = 2 + slen + 4;
  if (adler_out) *adler_out = adler;
  return ZT_OK;
}

int zt_zlib_decompress(const uint8_t *in, size_t n, size_t index, int verify, uint8_t **out, size_t *out_len,
                       size_t *end_ip, uint32_t *adler_out) {
  if (!out || !out_len) return set_error(ZT_E_ARG, "null output");
  if (n && !in) return set_error(ZT_E_ARG, "null input");
  Reader b{in, n, index};
  const int cmf = b.byte(), flg = b.byte();
  char msg[96];
  // src/Inflate.ts:44-58
  if (cmf < 0 || (cmf & 0x0F) != 8) return set_error(ZT_E_ZLIB_METHOD, "unsupported compression method");
  if (flg < 0) return set_error(ZT_E_ZLIB_FCHECK, "invalid fcheck flag:NaN");
  if (((cmf << 8) + flg) % 31 != 0) {
    snprintf(msg, sizeof msg, "invalid fcheck flag:%d", ((cmf << 8) + flg) % 31);
    return set_error(ZT_E_ZLIB_FCHECK, msg);
  }
  if (flg & 0x20) return set_error(ZT_E_ZLIB_FDICT, "fdict flag is not supported");
  uint8_t *o = nullptr;
  size_t olen = 0, eip = 0;
  ZT_TRY(zt_inflate_raw(in, n, b.p, nullptr, &o, &olen, &eip));
  uint32_t adler = 1;
  if (verify) {
    // src/Inflate.ts:80-90 (the Adler-32 of the output, on the GPU)
    const int rc = zt_adler32_update(1, o, olen, &adler);
    if (rc) {
      zt_free(o);
      return rc;
    }
    Reader t{in, n, eip};
    uint32_t want = 0;
    for (int k = 0; k < 4; ++k) want = (want << 8) | t.u8();
    if (adler != want) {
      zt_free(o);
      return set_error(ZT_E_ZLIB_ADLER, "invalid adler-32 checksum");
    }
  }
  *out = o;
  *out_len = olen;
  if (end_ip) *end_ip = eip;
  if (adler_out) *adler_out = adler;
  return ZT_OK;
}

}  // extern "C"
