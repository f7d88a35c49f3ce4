// zip_api.cpp -- Zip / Unzip archives over the batch engine (SURVEY.md 8(f)
// row 3; include/zt.h).  No ZipCrypto.
//
// zt_zip_compress follows src/Zip.ts:117-372: local file headers with the data,
// then the central directory and its end record, laid out byte for byte as the
// reference does.  Every DEFLATE member of the archive is compressed in one
// batch pipeline per device (batch_api.cpp) and every member's CRC-32 comes
// from the batched checksum kernel on the same device copy of the inputs.
// zt_unzip follows src/Unzip.ts:150-304: the end record is searched backwards,
// the central directory and the local headers are parsed with the reference's
// checks and messages, and every DEFLATE member is inflated in one batch (the
// two-phase batch inflate of inflate_api.cpp); `verify` checks each CRC-32 on
// the GPU.
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "zt_internal.h"

namespace zt {

int inflate_batch_dev_streams(DeviceCtx *c, const void *d_in, const std::vector<size_t> &in_off, const size_t *n,
                              const size_t *index, size_t count, uint8_t **out, size_t *out_len, size_t *end_ip,
                              int *status);

namespace {

void put16(std::vector<uint8_t> &o, uint32_t v) {
  o.push_back(v & 0xFF);
  o.push_back((v >> 8) & 0xFF);
}
void put32(std::vector<uint8_t> &o, uint32_t v) {
  for (int k = 0; k < 4; ++k) o.push_back((v >> (8 * k)) & 0xFF);
}

// little-endian reads as src/ByteStream.ts (bytes past the end read as 0 here;
// the reference reads `undefined`, which its comparisons reject the same way)
struct BS {
  const uint8_t *b;
  size_t n, p;
  int byte() { return p < n ? b[p++] : (++p, -1); }
  uint32_t u8() { return p < n ? b[p++] : (++p, 0u); }
  uint32_t u16() {
    const uint32_t a = u8();
    return a | (u8() << 8);
  }
  uint32_t u32() {
    const uint32_t a = u16();
    return a | (u16() << 16);
  }
};

}  // namespace
}  // namespace zt

using namespace zt;

extern "C" {

int zt_zip_compress(const uint8_t *const *in, const size_t *n, const zt_zip_file *files, size_t count,
                    const uint8_t *comment, size_t comment_len, uint8_t **out, size_t *out_len) {
  if (!out || !out_len) return set_error(ZT_E_ARG, "null output");
  if (count && (!in || !n || !files)) return set_error(ZT_E_ARG, "null argument");
  // DEFLATE members: one batch per deflate setting (normally one)
  std::vector<uint8_t *> body(count, nullptr);
  std::vector<size_t> blen(count, 0);
  std::vector<uint32_t> crc(count, 0);
  struct Freer {
    std::vector<uint8_t *> &v;
    ~Freer() {
      for (uint8_t *p : v) zt_free(p);
    }
  } freer{body};
  std::vector<size_t> defl, stored;
  for (size_t i = 0; i < count; ++i) {
    // only DEFLATE (8) is compressed; any other method number is stored
    // as-is and written unchanged into both headers (src/Zip.ts:92,146,255)
    (files[i].method == 8 ? defl : stored).push_back(i);
  }
  while (!defl.empty()) {
    const zt_deflate_opts o0 = files[defl[0]].deflate;
    std::vector<size_t> grp, rest;
    for (size_t i : defl) {
      const zt_deflate_opts &o = files[i].deflate;
      (o.compression_type == o0.compression_type && o.lazy == o0.lazy && o.level == o0.level ? grp : rest).push_back(i);
    }
    std::vector<const uint8_t *> pi(grp.size());
    std::vector<size_t> pn(grp.size()), olen(grp.size());
    std::vector<uint8_t *> po(grp.size(), nullptr);
    std::vector<int> st(grp.size());
    for (size_t k = 0; k < grp.size(); ++k) {
      pi[k] = in[grp[k]];
      pn[k] = n[grp[k]];
    }
    // GZip framing computes the CRC-32 beside the deflate on the same device bytes
    zt_gzip_opts go{};
    go.deflate = o0;
    const int rc = zt_gzip_compress_batch(pi.data(), pn.data(), grp.size(), &go, po.data(), olen.data(), st.data());
    if (rc) return rc;
    for (size_t k = 0; k < grp.size(); ++k) {
      const size_t i = grp[k];
      // member = 10-byte header | raw DEFLATE | CRC-32 | ISIZE
      body[i] = po[k];
      blen[i] = olen[k];
      const uint8_t *t = po[k] + olen[k] - 8;
      crc[i] = t[0] | (t[1] << 8) | (t[2] << 16) | ((uint32_t)t[3] << 24);
    }
    defl.swap(rest);
  }
  // STORE members: only their CRC-32 (batched on the device)
  if (!stored.empty()) {
    std::vector<const uint8_t *> pi(stored.size());
    std::vector<size_t> pn(stored.size());
    for (size_t k = 0; k < stored.size(); ++k) {
      pi[k] = in[stored[k]];
      pn[k] = n[stored[k]];
    }
    std::vector<uint32_t> c2(stored.size());
    ZT_TRY(zt_crc32_batch(pi.data(), pn.data(), stored.size(), c2.data()));
    for (size_t k = 0; k < stored.size(); ++k) crc[stored[k]] = c2[k];
  }
  // layout: src/Zip.ts:189-372
  std::vector<uint8_t> lo, cd;
  for (size_t i = 0; i < count; ++i) {
    const zt_zip_file &f = files[i];
    const uint8_t *data = f.method == 8 ? body[i] + 10 : in[i];
    const size_t dlen = f.method == 8 ? blen[i] - 18 : n[i];
    const uint32_t offset = (uint32_t)lo.size();
    // local file header
    lo.insert(lo.end(), {0x50, 0x4b, 0x03, 0x04});
    put16(lo, 20);                 // version needed
    put16(lo, 0);                  // flags
    put16(lo, (uint32_t)f.method);
    lo.insert(lo.end(), f.mtime, f.mtime + 4);
    put32(lo, crc[i]);
    put32(lo, (uint32_t)dlen);
    put32(lo, (uint32_t)n[i]);
    put16(lo, (uint32_t)f.name_len);
    put16(lo, 0);                  // extra field length
    if (f.name_len) lo.insert(lo.end(), f.name, f.name + f.name_len);
    if (dlen) lo.insert(lo.end(), data, data + dlen);
    // central directory file header
    cd.insert(cd.end(), {0x50, 0x4b, 0x01, 0x02});
    cd.push_back(20);              // version made by
    cd.push_back((uint8_t)f.os);
    put16(cd, 20);
    put16(cd, 0);
    put16(cd, (uint32_t)f.method);
    cd.insert(cd.end(), f.mtime, f.mtime + 4);
    put32(cd, crc[i]);
    put32(cd, (uint32_t)dlen);
    put32(cd, (uint32_t)n[i]);
    put16(cd, (uint32_t)f.name_len);
    put16(cd, 0);
    put16(cd, (uint32_t)f.comment_len);
    put16(cd, 0);                  // disk number start
    put16(cd, 0);                  // internal attributes
    put32(cd, 0);                  // external attributes
    put32(cd, offset);
    if (f.name_len) cd.insert(cd.end(), f.name, f.name + f.name_len);
    if (f.comment_len) cd.insert(cd.end(), f.comment, f.comment + f.comment_len);
  }
  std::vector<uint8_t> eo = {0x50, 0x4b, 0x05, 0x06, 0, 0, 0, 0};
  put16(eo, (uint32_t)count);
  put16(eo, (uint32_t)count);
  put32(eo, (uint32_t)cd.size());
  put32(eo, (uint32_t)lo.size());
  put16(eo, (uint32_t)comment_len);
  if (comment_len) eo.insert(eo.end(), comment, comment + comment_len);
  const size_t total = lo.size() + cd.size() + eo.size();
  uint8_t *h = host_out(total);
  if (!h) return set_error(ZT_E_NOMEM, "host allocation failed");
  memcpy(h, lo.data(), lo.size());
  memcpy(h + lo.size(), cd.data(), cd.size());
  memcpy(h + lo.size() + cd.size(), eo.data(), eo.size());
  *out = h;
  *out_len = total;
  return ZT_OK;
}

int zt_unzip(const uint8_t *in, size_t n, int verify, uint8_t **out, size_t *out_len, zt_unzip_entry **entries,
             size_t *count) {
  if (!out || !out_len || !entries || !count) return set_error(ZT_E_ARG, "null output");
  if (n && !in) return set_error(ZT_E_ARG, "null input");
  *out = nullptr;
  *entries = nullptr;
  *count = 0;
  // end of central directory: src/Unzip.ts:150-188 (backwards from n - 12)
  int64_t eo = -1;
  for (int64_t ip = (int64_t)n - 12; ip > 0; --ip)
    if (in[ip] == 0x50 && in[ip + 1] == 0x4b && in[ip + 2] == 0x05 && in[ip + 3] == 0x06) {
      eo = ip;
      break;
    }
  if (eo < 0) return set_error(ZT_E_ZIP_FORMAT, "End of Central Directory Record not found");
  BS b{in, n, (size_t)eo + 4};
  b.u16();                          // number of this disk
  b.u16();                          // start disk
  b.u16();                          // entries on this disk
  const uint32_t total = b.u16();   // total entries
  const uint32_t cd_size = b.u32();
  const uint32_t cd_off = b.u32();
  // central directory: src/Unzip.ts:78-130, 220-241
  std::vector<zt_unzip_entry> ent(total);
  BS c{in, n, cd_off};
  for (uint32_t i = 0; i < total; ++i) {
    zt_unzip_entry &e = ent[i];
    memset(&e, 0, sizeof e);
    if (c.byte() != 0x50 || c.byte() != 0x4b || c.byte() != 0x01 || c.byte() != 0x02)
      return set_error(ZT_E_ZIP_FORMAT, "invalid file header signature");
    e.version = c.u8();
    e.os = c.u8();
    e.need_version = c.u16();
    e.flags = c.u16();
    e.method = c.u16();
    e.time = c.u16();
    e.date = c.u16();
    e.crc32 = c.u32();
    e.compressed_size = c.u32();
    e.plain_size = c.u32();
    const uint32_t nl = c.u16(), xl = c.u16(), cl = c.u16();
    c.u16();  // disk number start
    c.u16();  // internal attributes
    c.u32();  // external attributes
    e.local_offset = c.u32();
    e.name_off = c.p;
    e.name_len = nl;
    c.p += nl + xl;
    e.comment_off = c.p;
    e.comment_len = cl;
    c.p += cl;
  }
  if ((uint64_t)cd_size < c.p - (uint64_t)cd_off) return set_error(ZT_E_ZIP_FORMAT, "invalid file header size");
  // local headers: src/Unzip.ts:28-62, 248-291
  std::vector<size_t> doff(total, 0), dlen(total, 0);
  std::vector<char> open_end(total, 0);
  std::vector<size_t> defl;
  for (uint32_t i = 0; i < total; ++i) {
    zt_unzip_entry &e = ent[i];
    BS l{in, n, e.local_offset};
    if (l.byte() != 0x50 || l.byte() != 0x4b || l.byte() != 0x03 || l.byte() != 0x04) {
      e.status = ZT_E_ZIP_FORMAT;
      snprintf(e.message, sizeof e.message, "invalid local file header signature");
      continue;
    }
    l.u16();                         // version needed
    const uint32_t flags = l.u16();
    const uint32_t method = l.u16();
    l.u16();
    l.u16();
    const uint32_t lcrc = l.u32();
    const uint32_t csize = l.u32();
    l.u32();
    const uint32_t nl = l.u16(), xl = l.u16();
    l.p += nl + xl;
    e.local_crc32 = lcrc;
    e.local_method = method;
    if (flags & 1) {
      e.status = ZT_E_ZIP_ENCRYPTED;
      snprintf(e.message, sizeof e.message, "encrypted: please set password");
      continue;
    }
    doff[i] = l.p;
    dlen[i] = csize;
    // a data descriptor (flag bit 3) leaves the local size 0: such a member's
    // stream is bounded by nothing before the input's end, as in the
    // reference's RawInflate from the member's offset (src/Unzip.ts:284-288)
    open_end[i] = (flags & 8) != 0 || csize == 0;
    if (method == 8) defl.push_back(i);
  }
  // every DEFLATE member inflated in one batch (RawInflate from the member's
  // offset over the whole input, src/Unzip.ts:284-288)
  std::vector<uint8_t *> o(total, nullptr);
  std::vector<size_t> ol(total, 0);
  struct Freer {
    std::vector<uint8_t *> &v;
    ~Freer() {
      for (uint8_t *p : v) zt_free(p);
    }
  } freer{o};
  if (!defl.empty()) {
    DeviceCtx *dc;
    ZT_TRY(get_ctx(&dc));
    std::lock_guard<std::recursive_mutex> ctx_lock(dc->mu);
    void *d_in;
    ZT_TRY(scratch(dc, 19, n + 64, &d_in));
    ZT_TRY(upload(dc, d_in, in, n, dc->stream));
    const size_t m = defl.size();
    // (a member with a known compressed size reads at most 64 KiB past it:
    // a valid stream ends inside, and only a corrupt one would read on into
    // the next bytes.  A member without one -- data descriptor -- is first
    // bounded by the next local header in file order (or the central
    // directory) + 64 KiB, so that the batch's per-stream scratch stays
    // proportional to the archive; only members that fail inside that bound
    // are decoded again over the rest of the input, as the reference's
    // RawInflate from the member's offset would read it.)
    std::vector<size_t> starts;
    for (uint32_t i = 0; i < total; ++i) starts.push_back(ent[i].local_offset);
    starts.push_back(cd_off);
    std::sort(starts.begin(), starts.end());
    std::vector<size_t> in_off(m, 0), nn(m, n), idx(m), bl(m), eip(m);
    std::vector<uint8_t *> bp(m, nullptr);
    Freer bp_freer{bp};  // (every early return frees what the batch allocated; handed-on pointers are nulled)
    // (a batch that fails as a whole -- device memory, HIP -- leaves kNotRun)
    constexpr int kNotRun = -0x7FFF;
    std::vector<int> st(m, kNotRun);
    std::vector<char> bounded(m, 0);
    for (size_t k = 0; k < m; ++k) {
      const size_t i = defl[k];
      idx[k] = std::min(doff[i], n);
      if (open_end[i]) {
        const auto nx = std::upper_bound(starts.begin(), starts.end(), (size_t)ent[i].local_offset);
        if (nx != starts.end() && *nx >= idx[k]) {
          nn[k] = std::min<size_t>(n, *nx + (64u << 10));
          bounded[k] = nn[k] < n;
        }
      } else {
        nn[k] = std::min<size_t>(n, idx[k] + dlen[i] + (64u << 10));
      }
    }
    int rc = inflate_batch_dev_streams(dc, d_in, in_off, nn.data(), idx.data(), m, bp.data(), bl.data(),
                                       eip.data(), st.data());
    for (size_t k = 0; k < m; ++k)
      if (st[k] == kNotRun) return rc ? rc : set_error(ZT_E_INTERNAL, "unzip: member batch not decoded");
    // members that failed inside their bound: again, to the input's end
    std::vector<size_t> again;
    for (size_t k = 0; k < m; ++k)
      if (st[k] && bounded[k]) again.push_back(k);
    if (!again.empty()) {
      const size_t r = again.size();
      std::vector<size_t> in2(r, 0), nn2(r, n), idx2(r), bl2(r), eip2(r);
      std::vector<uint8_t *> bp2(r, nullptr);
      std::vector<int> st2(r, kNotRun);
      for (size_t j = 0; j < r; ++j) idx2[j] = idx[again[j]];
      rc = inflate_batch_dev_streams(dc, d_in, in2, nn2.data(), idx2.data(), r, bp2.data(), bl2.data(), eip2.data(),
                                     st2.data());
      for (size_t j = 0; j < r; ++j)
        if (st2[j] == kNotRun) {
          for (uint8_t *p : bp2) zt_free(p);
          return rc ? rc : set_error(ZT_E_INTERNAL, "unzip: member batch not decoded");
        }
      for (size_t j = 0; j < r; ++j) {
        const size_t k = again[j];
        zt_free(bp[k]);
        bp[k] = bp2[j];
        bl[k] = bl2[j];
        st[k] = st2[j];
      }
    }
    for (size_t k = 0; k < m; ++k) {
      const size_t i = defl[k];
      if (st[k]) {
        ent[i].status = st[k];
        inflate_error(st[k], 0);
        snprintf(ent[i].message, sizeof ent[i].message, "%s", zt_last_error_message());
        zt_free(bp[k]);
        bp[k] = nullptr;
        continue;
      }
      o[i] = bp[k];
      bp[k] = nullptr;
      ol[i] = bl[k];
    }
  }
  // STORE members: the compressed-size bytes after the local header
  for (uint32_t i = 0; i < total; ++i) {
    if (ent[i].status || ent[i].local_method == 8) continue;
    const size_t a = std::min(doff[i], n), len = std::min(dlen[i], n - a);
    o[i] = (uint8_t *)malloc(len ? len : 1);
    if (!o[i]) return set_error(ZT_E_NOMEM, "host allocation failed");
    if (len) memcpy(o[i], in + a, len);
    ol[i] = len;
  }
  // the output: every entry's data, concatenated
  size_t tot = 0;
  for (uint32_t i = 0; i < total; ++i) tot += ol[i];
  uint8_t *h = host_out(tot);
  if (!h) return set_error(ZT_E_NOMEM, "host allocation failed");
  size_t p = 0;
  std::vector<const uint8_t *> cp;
  std::vector<size_t> cn;
  for (uint32_t i = 0; i < total; ++i) {
    ent[i].data_off = p;
    ent[i].data_len = ol[i];
    if (ol[i]) memcpy(h + p, o[i], ol[i]);
    p += ol[i];
    cp.push_back(h + ent[i].data_off);
    cn.push_back(ol[i]);
  }
  // CRC-32 of every entry's data (batched on the device): src/Unzip.ts:293-301
  std::vector<uint32_t> dcrc(total, 0);
  if (total) {
    const int rc = zt_crc32_batch(cp.data(), cn.data(), total, dcrc.data());
    if (rc) {
      zt_free(h);
      return rc;
    }
  }
  for (uint32_t i = 0; i < total; ++i) {
    ent[i].data_crc32 = dcrc[i];
    if (verify && !ent[i].status && dcrc[i] != ent[i].local_crc32) {
      ent[i].status = ZT_E_ZIP_CRC;
      snprintf(ent[i].message, sizeof ent[i].message, "Incorrect crc: file=0x%x, data=0x%x", ent[i].local_crc32,
               dcrc[i]);
    }
  }
  zt_unzip_entry *E = (zt_unzip_entry *)malloc((total ? total : 1) * sizeof(zt_unzip_entry));
  if (!E) {
    zt_free(h);
    return set_error(ZT_E_NOMEM, "host allocation failed");
  }
  if (total) memcpy(E, ent.data(), total * sizeof(zt_unzip_entry));
  *out = h;
  *out_len = tot;
  *entries = E;
  *count = total;
  for (uint32_t i = 0; i < total; ++i)
    if (ent[i].status) return set_error(ent[i].status, ent[i].message);
  return ZT_OK;
}

}  // extern "C"
