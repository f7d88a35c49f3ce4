// inflate_api.cpp -- host side of the inflate entry points (include/zt.h).
#include <algorithm>
#include <cstdio>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "zt_internal.h"

namespace zt {


// Message text of the reference for each status (src/RawInflate.ts).
int inflate_error(int status, int detail) {
  char buf[96];
  switch (status) {
    case ZT_E_INPUT_BROKEN: return set_error(status, "input buffer is broken");
    case ZT_E_INVALID_CODE_LENGTH:
      snprintf(buf, sizeof buf, "invalid code length: %d", detail);
      return set_error(status, buf);
    case ZT_E_UNKNOWN_BTYPE:
      snprintf(buf, sizeof buf, "unknown BTYPE: %d", detail);
      return set_error(status, buf);
    case ZT_E_STORED_LEN: return set_error(status, "invalid uncompressed block header: LEN");
    case ZT_E_STORED_NLEN: return set_error(status, "invalid uncompressed block header: NLEN");
    case ZT_E_INVALID_DISTANCE: return set_error(status, "invalid distance too far back");
    case ZT_E_INVALID_SYMBOL: return set_error(status, "invalid literal/length or distance code");
    case ZT_E_BAD_TREE: return set_error(status, "invalid code lengths set");
    default: return set_error(status, "inflate failed");
  }
}

static size_t align_up(size_t v, size_t a) { return (v + a - 1) / a * a; }

// Two-phase batch decode (inflate_tok.hip applied per stream): one tokenize
// wave per stream (no history ring in LDS, so many streams per CU), then
// expand + copy with one segment per stream, all outputs in one buffer.
// Streams it cannot finish (errors, a token overflow, an empty input) are
// appended to `failed` for the one-wave decoder, which also yields the
// reference's exact error. Outputs of the others are malloc'd and filled.
// ZT_BATCH_TIMING=1: host wall time of the batch stages on stderr (measurement only)
static double bt_now() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
static bool bt_on() {
  static const bool on = getenv("ZT_BATCH_TIMING") != nullptr;
  return on;
}
#define BT(label) \
  if (bt_on()) fprintf(stderr, "[batch] %-28s %8.2f ms\n", label, bt_now())

static int batch_two_phase(DeviceCtx *c, const uint8_t *d_in, const std::vector<size_t> &in_off, const size_t *n,
                           const size_t *index, size_t count, uint8_t **out, size_t *out_len,
                           std::vector<InfResult> &res, std::vector<size_t> &failed) {
  hipStream_t s = c->stream;
  std::vector<size_t> ids;
  for (size_t i = 0; i < count; ++i) {
    const size_t st = index ? index[i] : 0;
    if (n[i] > st)
      ids.push_back(i);
    else
      failed.push_back(i);
  }
  if (ids.empty()) return ZT_OK;
  // longest input first: one wave per stream, and workgroups go to the 8 XCDs
  // round robin -- a batch alternating slow and fast streams (C2: random-data
  // and text blocks) would otherwise put every slow one on half of the XCDs
  std::stable_sort(ids.begin(), ids.end(), [&](size_t a, size_t b) {
    return n[a] - (index ? index[a] : 0) > n[b] - (index ? index[b] : 0);
  });
  const size_t units = ids.size();
  std::vector<TokJob> jobs(units);
  uint64_t tok_total = 0;
  for (size_t k = 0; k < units; ++k) {
    const size_t i = ids[k];
    TokJob &j = jobs[k];
    j.start = in_off[i] + (index ? index[i] : 0);
    j.end = in_off[i] + n[i];
    // tokens <= output bytes; every token takes >= 1 input bit
    uint64_t cap = std::max<uint64_t>(65536, 4 * (uint64_t)(n[i] - (index ? index[i] : 0)));
    cap = std::min<uint64_t>(cap, (j.end - j.start) * 8) + 64;
    // (TokResult::ntok carries flags in bits 30-31: a full slot must not reach them)
    cap = std::min<uint64_t>(cap, (1u << 30) - 64);
    j.tok_off = tok_total;
    j.tok_cap = (uint32_t)cap;
    j.stop_first = 0;
    tok_total += align_up(cap, 64);
  }
  void *d_tok, *d_meta;
  ZT_TRY(scratch(c, 4, (tok_total + 256) * 4, &d_tok));  // + slack: chunked token reads
  const size_t jobs_bytes = align_up(units * sizeof(TokJob), 256);
  ZT_TRY(scratch(c, 6, jobs_bytes + align_up(units * sizeof(TokResult), 256), &d_meta));
  TokJob *d_jobs = static_cast<TokJob *>(d_meta);
  TokResult *d_tres = reinterpret_cast<TokResult *>(static_cast<uint8_t *>(d_meta) + jobs_bytes);
  ZT_HIP(hipMemcpyAsync(d_jobs, jobs.data(), units * sizeof(TokJob), hipMemcpyHostToDevice, s));
  TokParams tp{};
  tp.in = d_in;
  tp.n = 0;
  tp.stops = reinterpret_cast<const uint64_t *>(d_meta);  // never read: nstops = 0
  tp.nstops = 0;
  tp.jobs = d_jobs;
  tp.res = d_tres;
  tp.tokens = static_cast<uint32_t *>(d_tok);
  tp.count = (uint32_t)units;
  static const char *simt_env = getenv("ZT_TOK_SIMT");  // (A/B: 0 = one-lane body decode)
  tp.simt = simt_env ? atoi(simt_env) != 0 : 1;
  tp.dbg = nullptr;
  tp.dump_unit = 0xFFFFFFFFu;
  tp.dump_once = 0;
  tp.run_tokens = 1;
  BT("tokenize launch");
  ZT_TRY(tokenize_units_dev(tp, s));
  std::vector<TokResult> tr(units);
  ZT_TRY(readback(c, tr.data(), d_tres, units * sizeof(TokResult), s));
  BT("tokenize done");
  // one chain unit and one segment per stream that decoded to BFINAL
  std::vector<ChainUnit> chain;
  std::vector<SegJob> segs;
  std::vector<size_t> who;
  uint64_t out_total = 0, desc_total = 0;
  for (size_t k = 0; k < units; ++k) {
    const TokResult &r = tr[k];
    if (r.status != ZT_OK || r.stop_idx >= 0 || r.out_len > 0xFFFFFFFFull) {
      failed.push_back(ids[k]);
      continue;
    }
    desc_total = align_up(desc_total, 512);
    // (a stream of stored runs only: expand_kernel writes it straight from
    // the input, copy_kernel skips its segment -- inflate_seg.hip)
    const bool direct = (r.ntok >> 30) == 3u;
    segs.push_back(SegJob{(uint32_t)chain.size(), direct ? 0x80000001u : 1u});
    chain.push_back(ChainUnit{jobs[k].tok_off, out_total, out_total, desc_total, r.ntok, (uint32_t)r.out_len});
    who.push_back(k);
    out_total += align_up(r.out_len ? r.out_len : 1, 256);
    desc_total += r.out_len;
  }
  if (chain.empty()) return ZT_OK;
  void *d_out, *d_chain, *d_desc;
  ZT_TRY(scratch(c, 1, out_total, &d_out));
  const size_t chain_bytes = align_up(chain.size() * sizeof(ChainUnit), 256);
  const size_t seg_bytes = align_up(segs.size() * sizeof(SegJob), 256);
  const size_t ust_bytes = align_up(chain.size() * 4, 256);
  ZT_TRY(scratch(c, 7, chain_bytes + seg_bytes + 2 * ust_bytes, &d_chain));
  ZT_TRY(scratch(c, 3, (desc_total + 1024) * 2, &d_desc));  // + slack: chunked descriptor reads
  ChainUnit *d_cu = static_cast<ChainUnit *>(d_chain);
  SegJob *d_sj = reinterpret_cast<SegJob *>(static_cast<uint8_t *>(d_chain) + chain_bytes);
  int32_t *d_ust = reinterpret_cast<int32_t *>(static_cast<uint8_t *>(d_chain) + chain_bytes + seg_bytes);
  int32_t *d_st = reinterpret_cast<int32_t *>(static_cast<uint8_t *>(d_chain) + chain_bytes + seg_bytes + ust_bytes);
  ZT_HIP(hipMemcpyAsync(d_cu, chain.data(), chain.size() * sizeof(ChainUnit), hipMemcpyHostToDevice, s));
  ZT_HIP(hipMemcpyAsync(d_sj, segs.data(), segs.size() * sizeof(SegJob), hipMemcpyHostToDevice, s));
  ResolveParams rp;
  rp.tokens = static_cast<const uint32_t *>(d_tok);
  rp.units = d_cu;
  rp.segs = d_sj;
  rp.out = static_cast<uint8_t *>(d_out);
  rp.desc = static_cast<uint16_t *>(d_desc);
  rp.unit_status = d_ust;
  rp.seg_status = d_st;
  rp.nunits = (uint32_t)chain.size();
  rp.nseg = (uint32_t)segs.size();
  rp.marker = 0;
  rp.in = d_in;
  ZT_TRY(resolve_segments_dev(rp, s));
  std::vector<int32_t> ust(chain.size()), sst(segs.size());
  ZT_HIP(hipMemcpyAsync(ust.data(), d_ust, chain.size() * 4, hipMemcpyDeviceToHost, s));
  ZT_HIP(hipMemcpyAsync(sst.data(), d_st, segs.size() * 4, hipMemcpyDeviceToHost, s));
  ZT_HIP(hipStreamSynchronize(s));
  BT("resolve done");
  std::vector<size_t> done;
  for (size_t j = 0; j < chain.size(); ++j)
    if (ust[j] == ZT_OK && sst[j] == ZT_OK) done.push_back(j);
  if (!done.empty()) {
    // The finished outputs share one slab (slab_out) laid out as the device
    // output (items at their 256-aligned offsets), so one download fills it;
    // the slab comes from the host output pool -- registered once its items
    // are freed -- and a registered one takes the DMA directly (the staged
    // download and a copy-out into a fresh slab cost ~7 ms per 256 MiB, C2)
    uint8_t *slab = slab_out(out_total, done.size(), true);
    if (!slab) return set_error(ZT_E_NOMEM, "host allocation failed");
    if (const int rc = download(c, slab, d_out, out_total, s)) {
      for (size_t q = 0; q < done.size(); ++q) slab_release(slab);
      return rc;
    }
    for (const size_t j : done) {
      const size_t k = who[j], i = ids[k];
      out[i] = slab + chain[j].out_off;
      out_len[i] = chain[j].out_len;
      InfResult &r = res[i];
      r = InfResult{};
      r.out_len = chain[j].out_len;
      r.end_ip = ((tr[k].end_bits + 7) >> 3) - in_off[i];
      r.status = ZT_OK;
      r.stop_idx = -1;
    }
  }
  for (size_t j = 0; j < chain.size(); ++j)
    if (ust[j] != ZT_OK || sst[j] != ZT_OK) failed.push_back(ids[who[j]]);
  BT("download done");
  return ZT_OK;
}

// Decode `count` device-resident streams (stream i at d_in + in_off[i],
// n[i] bytes, from index[i]); outputs are malloc'd.
int inflate_batch_dev_streams(DeviceCtx *c, const void *d_in, const std::vector<size_t> &in_off, const size_t *n,
                              const size_t *index, size_t count, uint8_t **out, size_t *out_len, size_t *end_ip,
                              int *status);
static int inflate_dev_batch(DeviceCtx *c, const void *d_in, const std::vector<size_t> &in_off, const size_t *n,
                             const size_t *index, size_t count, int strict, uint8_t **out, size_t *out_len,
                             size_t *end_ip, int *status) {
  std::vector<size_t> cap(count);
  for (size_t i = 0; i < count; ++i) {
    // first guess (4x the stream's bytes from its start); exact sizes are
    // known after one pass
    size_t g = 4 * (n[i] - std::min(n[i], index ? index[i] : (size_t)0));
    cap[i] = g < 65536 ? 65536 : g;
  }
  void *d_jobs, *d_res;
  ZT_TRY(scratch(c, 2, count * (sizeof(InfJob) + sizeof(InfResult)) + 256, &d_jobs));
  d_res = (uint8_t *)d_jobs + align_up(count * sizeof(InfJob), 256);
  std::vector<InfJob> jobs(count);
  std::vector<InfResult> res(count);
  std::vector<size_t> todo;
  // non-strict batches of several streams: two-phase first, one wave per
  // stream for whatever it leaves (ZT_BATCH_ONEWAVE=1 forces the latter)
  static const bool onewave = getenv("ZT_BATCH_ONEWAVE") != nullptr;
  if (!strict && count >= 8 && !onewave) {
    ZT_TRY(batch_two_phase(c, (const uint8_t *)d_in, in_off, n, index, count, out, out_len, res, todo));
    std::sort(todo.begin(), todo.end());
  } else {
    todo.resize(count);
    for (size_t i = 0; i < count; ++i) todo[i] = i;
  }
  for (int pass = 0; pass < 2 && !todo.empty(); ++pass) {
    // (one wave per stream)
    size_t out_total = 0;
    std::vector<size_t> out_off(todo.size());
    for (size_t k = 0; k < todo.size(); ++k) {
      out_off[k] = out_total;
      out_total += align_up(cap[todo[k]], 256);
    }
    void *d_out;
    ZT_TRY(scratch(c, 1, out_total, &d_out));
    for (size_t k = 0; k < todo.size(); ++k) {
      size_t i = todo[k];
      jobs[k] = InfJob{};
      jobs[k].in = (const uint8_t *)d_in + in_off[i];
      jobs[k].n = n[i];
      jobs[k].start = index ? index[i] : 0;
      jobs[k].out = (uint8_t *)d_out + out_off[k];
      jobs[k].cap = cap[i];
      jobs[k].strict = strict;
    }
    ZT_HIP(hipMemcpyAsync(d_jobs, jobs.data(), todo.size() * sizeof(InfJob), hipMemcpyHostToDevice, c->stream));
    ZT_TRY(inflate_jobs_dev((const InfJob *)d_jobs, (InfResult *)d_res, (int)todo.size(), c->stream));
    if (pass == 0) c->times.inflate_paths[2] += todo.size();
    std::vector<InfResult> r(todo.size());
    ZT_TRY(readback(c, r.data(), d_res, todo.size() * sizeof(InfResult), c->stream));
    std::vector<size_t> again, done;
    // finished outputs are packed on the device side already (out_off);
    // one D2H of the span up to the last finished byte into pinned staging
    size_t span = 0;
    for (size_t k = 0; k < todo.size(); ++k) {
      size_t i = todo[k];
      res[i] = r[k];
      if (r[k].status == ZT_OK && r[k].out_len > cap[i]) {
        cap[i] = r[k].out_len;  // rerun with the exact size
        again.push_back(i);
        continue;
      }
      out[i] = nullptr;
      out_len[i] = 0;
      if (r[k].status == ZT_OK) {
        out[i] = (uint8_t *)malloc(r[k].out_len ? r[k].out_len : 1);
        if (!out[i]) return set_error(ZT_E_NOMEM, "host allocation failed");
        out_len[i] = r[k].out_len;
        done.push_back(k);
        if (out_off[k] + r[k].out_len > span) span = out_off[k] + r[k].out_len;
      }
    }
    if (span) {
      void *h;
      ZT_TRY(pinned(c, span, &h));
      const uint8_t *stage = (const uint8_t *)h;
      ZT_HIP(hipMemcpyAsync(h, d_out, span, hipMemcpyDeviceToHost, c->stream));
      ZT_HIP(hipStreamSynchronize(c->stream));
      parallel_copy(done.size(), [&](size_t j) {
        const size_t k = done[j], i = todo[k];
        if (out_len[i]) memcpy(out[i], stage + out_off[k], out_len[i]);
      }, span);
    }
    todo.swap(again);
  }
  int first = ZT_OK;
  for (size_t i = 0; i < count; ++i) {
    status[i] = res[i].status;
    if (end_ip) end_ip[i] = res[i].end_ip;
    if (status[i] && first == ZT_OK) first = inflate_error(res[i].status, res[i].detail);
  }
  return first;
}

int inflate_batch_dev_streams(DeviceCtx *c, const void *d_in, const std::vector<size_t> &in_off, const size_t *n,
                              const size_t *index, size_t count, uint8_t **out, size_t *out_len, size_t *end_ip,
                              int *status) {
  return inflate_dev_batch(c, d_in, in_off, n, index, count, 0, out, out_len, end_ip, status);
}

// Decode `count` host streams; outputs are malloc'd.
static int inflate_host_batch(const uint8_t *const *in, const size_t *n, const size_t *index, size_t count,
                              const zt_inflate_opts *opts, uint8_t **out, size_t *out_len, size_t *end_ip,
                              int *status) {
  DeviceCtx *c;
  ZT_TRY(get_ctx(&c));
  std::lock_guard<std::recursive_mutex> ctx_lock(c->mu);
  const int strict = opts ? opts->ref_strict : 0;
  std::vector<size_t> in_off(count);
  size_t in_total = 0;
  for (size_t i = 0; i < count; ++i) {
    in_off[i] = in_total;
    in_total += align_up(n[i] ? n[i] : 1, 256);
  }
  void *d_in;
  ZT_TRY(scratch(c, 0, in_total, &d_in));
  // inputs packed into pinned staging in chunks of about 32 MiB, each
  // chunk's upload issued as soon as it is packed: the copy engine moves
  // chunk k while the host packs chunk k + 1 (C2: pack 2.0 ms, then H2D 2.8)
  {
    void *h;
    ZT_TRY(pinned(c, in_total, &h));
    uint8_t *stage = (uint8_t *)h;
    BT("pack start");
    constexpr size_t kChunk = 32u << 20;
    for (size_t a = 0; a < count;) {
      size_t b = a + 1;
      while (b < count && in_off[b] - in_off[a] < kChunk) ++b;
      const size_t lo = in_off[a], hi = b < count ? in_off[b] : in_total;
      // (every chunk with the whole batch's copy threads)
      parallel_copy(b - a, [&](size_t k) { copy_to_staging(stage + in_off[a + k], in[a + k], n[a + k]); }, in_total);
      ZT_HIP(hipMemcpyAsync((uint8_t *)d_in + lo, stage + lo, hi - lo, hipMemcpyHostToDevice, c->stream));
      a = b;
    }
    BT("pack done");
  }
  return inflate_dev_batch(c, d_in, in_off, n, index, count, strict, out, out_len, end_ip, status);
}

// One device-resident stream from `index` (gzip / zlib members): the
// segment-parallel and general paths scan a window that grows 8x at a time
// (a member's decode never scans the members after it, so many small members
// stay linear), then the one-wave decoder.  Output malloc'd.
int inflate_dev_member(DeviceCtx *c, const uint8_t *d_in, size_t n, size_t index, uint8_t **out, size_t *out_len,
                       size_t *end_ip) {
  hipStream_t s = c->stream;
  if (n >= index + (1u << 14)) {
    for (size_t w = 4u << 20;; w *= 8) {
      const size_t ne = std::min(n, index + w);
      uint8_t *d_out = nullptr;
      size_t ol = 0, eip = 0;
      int seg = inflate_segments_dev(c, d_in, ne, index, &d_out, 0, &ol, &eip, s);
      // the window cut a stream with sync points short (2): grow it, no
      // general-path attempt (it cannot finish inside the window either)
      if (seg == 2 && ne < n) continue;
      if (seg >= 1) seg = inflate_general_dev(c, d_in, ne, index, &d_out, 0, &ol, &eip, s);
      if (seg < 0) return seg;
      if (seg == 0) {
        uint8_t *h = host_out(ol);
        if (!h) return set_error(ZT_E_NOMEM, "host allocation failed");
        const int rc = download(c, h, d_out, ol, s);
        if (rc) {
          zt_free(h);
          return rc;
        }
        *out = h;
        *out_len = ol;
        *end_ip = eip;
        return ZT_OK;
      }
      if (ne == n) break;
    }
  }
  std::vector<size_t> in_off(1, 0);
  int st = 0;
  return inflate_dev_batch(c, d_in, in_off, &n, &index, 1, 0, out, out_len, end_ip, &st);
}

// Large host streams with restart points (this engine's deflate output, SURVEY
// 8(f)): PCIe overlapped with the decode, as deflate_raw_pipelined does for
// deflate.  The input is cut after restart markers (00 00 00 FF FF 00 00 00
// FF FF: empty stored blocks, no match reaches behind them) found by the host
// near every kInfPiece-th byte; piece i + 1 is uploaded while piece i is
// decoded and piece i - 1's bytes come back (pipeline_h2d_d2h).  A non-final
// piece gets an empty final stored block (01 00 00 FF FF) after it on the
// device and is decoded as a stream of its own: it must end exactly there,
// and a unit of its segment chain must start at the cut.  The second is the
// certificate that the cut is a real block boundary: the piece's decode
// starts at a true block start (induction from the stream start), so a
// block boundary exactly at the cut is the whole stream's boundary too --
// ending on the appended block alone is not (a crafted Huffman block can
// decode those five bytes as codes ending in EOB).  A piece whose
// matches reach behind its start fails in the segment decoder.  Any failure
// -- no marker, a piece the segment path cannot decode or certify --
// returns 1 and the caller decodes the whole stream in one call
// (tests/test_gpu_api_pipeline.py: identical output and end position).
static constexpr size_t kInfPipeMin = 32u << 20;
static constexpr size_t kInfPiece = 64u << 20;

static int inflate_raw_pipelined(DeviceCtx *c, const uint8_t *in, size_t n, size_t index, uint8_t **out,
                                 size_t *out_len, size_t *end_ip) {
  static const uint8_t kMarker[10] = {0, 0, 0, 0xFF, 0xFF, 0, 0, 0, 0xFF, 0xFF};
  static const uint8_t kFinal[5] = {1, 0, 0, 0xFF, 0xFF};
  const size_t m = n - index;
  // tuning hook: ZT_INF_PIECES = pieces per stream (default 8; each piece's
  // decode pays a few host round trips, so fewer, larger pieces)
  static const int np_env = getenv("ZT_INF_PIECES") ? atoi(getenv("ZT_INF_PIECES")) : 0;
  const size_t piece = std::min(std::max(m / (np_env > 1 ? np_env : 8), (size_t)8 << 20), kInfPiece);
  // tuning hook ZT_INF_RAMP = r: the first pieces ramp up (piece >> r, then
  // >> r - 1, ...) so that the downloads -- the pipeline's bound -- start
  // earlier; default 0: r = 2 measured 26.5 against 26.9 ms, within the
  // box's run-to-run spread (`gpurun_out/r06pc2`)
  static const int ramp = getenv("ZT_INF_RAMP") ? atoi(getenv("ZT_INF_RAMP")) : 0;
  auto target = [&](size_t k) { return piece >> (k < (size_t)ramp ? (size_t)ramp - k : 0); };
  std::vector<size_t> cut{index};
  for (size_t t = index + target(0); t + piece / 2 < n; t = cut.back() + target(cut.size() - 1)) {
    const size_t lo = std::max(t, cut.back()) - 10, hi = std::min(n, t + (8u << 20));
    const void *q = memmem(in + lo, hi - lo, kMarker, sizeof kMarker);
    if (!q) break;
    const size_t p = (size_t)((const uint8_t *)q - in) + sizeof kMarker;
    if (p + piece / 2 >= n) break;  // (the last piece keeps at least half a piece)
    cut.push_back(p);
  }
  cut.push_back(n);
  const size_t np = cut.size() - 1;
  if (np < 2) return 1;
  void *d_in;
  ZT_TRY(scratch(c, 0, m + 64 * np + 256, &d_in));
  // Results go to one device buffer at consecutive offsets (scratch slot 22,
  // 4x the input, as the host output used to be), each piece's capacity 4x
  // its input or what is left, and a piece that reports needing more is
  // decoded again with that.  Past the buffer's end (streams compressed
  // better than 4:1) the pieces go to a ring of 3 overflow buffers (slots
  // 23-25), piece i's once piece i - 3's bytes have left the device
  // (PipeOut::drain).  The host output starts at piece 0's ratio x the
  // stream and grows the same way (pipeline_h2d_d2h), so a stream of any
  // ratio stays pipelined.
  constexpr size_t kRing = 3;
  auto d_piece = [&](size_t i) { return (uint8_t *)d_in + (cut[i] - index) + 64 * i; };
  const size_t cap = std::max<size_t>(4 * m, 64u << 20);
  void *d_big;
  ZT_TRY(scratch(c, 22, cap, &d_big));
  size_t off = 0;      // bytes of the big buffer used
  size_t ring0 = np;   // first piece in the overflow ring
  double ratio0 = 0;   // output bytes per input byte of piece 0
  size_t eip_last = 0;
  PipeOut po;
  po.cap_fn = [&] { return (size_t)(ratio0 * 1.25 * (double)m) + (16u << 20); };
  auto compute = [&](size_t i, const void **d_res, size_t *n_res) -> int {
        const size_t len = cut[i + 1] - cut[i];
        const bool last = i + 1 == np;
        if (!last) {  // (by a kernel: no copy-engine command queued behind the pipeline's transfers)
          uint64_t fin = 0;
          for (int k = 0; k < (int)sizeof kFinal; ++k) fin |= (uint64_t)kFinal[k] << (8 * k);
          ZT_TRY(q_bytes(d_piece(i) + len, fin, (uint32_t)sizeof kFinal, c->stream));
        }
        const size_t pn = last ? len : len + sizeof kFinal;
        size_t want = 4 * pn + (1u << 20);
        if (i > 0) want = std::max(want, (size_t)(ratio0 * 1.25 * (double)pn) + (1u << 20));
        for (int attempt = 0; attempt < 2; ++attempt) {
          uint8_t *d_o;
          size_t ocap;
          // (first try: whatever room is left, at least 1 MiB; again: all it needs)
          if (i < ring0 && (attempt == 0 ? off + (1u << 20) <= cap : off + want <= cap)) {
            d_o = static_cast<uint8_t *>(d_big) + off;
            ocap = std::min(want, cap - off);
          } else {  // the overflow ring
            if (ring0 == np) ring0 = po.drain_from = i;
            const size_t r = (i - ring0) % kRing;
            if (i - ring0 >= kRing) ZT_TRY(po.drain(i - kRing));
            void *p;
            ZT_TRY(scratch(c, 23 + (int)r, want, &p));
            d_o = static_cast<uint8_t *>(p);
            ocap = want;  // (the capacity asked: the device chain sizes its descriptors from it)
          }
          size_t ol = 0, eip = 0;
          // a non-final piece must have a block boundary right before its
          // appended final block (the cut) -- and must end on that block
          int seg = inflate_segments_dev(c, d_piece(i), pn, 0, &d_o, ocap, &ol, &eip, c->stream, last ? ~0ull : len);
          if (seg < 0 && ol > ocap && attempt == 0) {  // more output than its room: again with what it needs
            want = ol;
            continue;
          }
          // (no sync points in the last piece: the speculative general decoder)
          if (seg >= 1 && last) seg = inflate_general_dev(c, d_piece(i), pn, 0, &d_o, ocap, &ol, &eip, c->stream);
          if (seg != 0) return seg < 0 ? seg : set_error(ZT_E_INTERNAL, "pipelined inflate: piece not decoded");
          if (!last && eip != pn) return set_error(ZT_E_INTERNAL, "pipelined inflate: a cut is not a block boundary");
          if (i == 0) ratio0 = (double)ol / (double)pn;
          if (i < ring0) off += (ol + 255) & ~(size_t)255;
          eip_last = eip;
          *d_res = d_o;
          *n_res = ol;
          return ZT_OK;
        }
        return set_error(ZT_E_INTERNAL, "pipelined inflate: piece output did not settle");
      };
  auto input = [&](size_t i) { return PipePiece{in + cut[i], d_piece(i), cut[i + 1] - cut[i]}; };
  const int rc = pipeline_h2d_d2h(c, np, input, compute, po);
  if (rc) {  // (every copy has finished: the buffer can go)
    host_discard(po.base);
    return 1;
  }
  host_out_used(po.base, po.total);
  *out = po.base;
  *out_len = po.total;
  if (end_ip) *end_ip = cut[np - 1] + eip_last;
  return ZT_OK;
}

}  // namespace zt

using namespace zt;

extern "C" {

int zt_inflate_raw(const uint8_t *in, size_t n, size_t index, const zt_inflate_opts *opts, uint8_t **out,
                   size_t *out_len, size_t *end_ip) {
  if (!out || !out_len) return set_error(ZT_E_ARG, "null output");
  if (!(opts && opts->ref_strict) && in && n >= index + (1u << 14)) {
    // large stream: segment-parallel decode when it carries restart points
    DeviceCtx *c;
    ZT_TRY(get_ctx(&c));
    std::lock_guard<std::recursive_mutex> ctx_lock(c->mu);
    static const bool no_pipe = getenv("ZT_INF_NOPIPE") != nullptr;  // (A/B measurement and the identity test)
    if (!no_pipe && n - index >= kInfPipeMin && inflate_raw_pipelined(c, in, n, index, out, out_len, end_ip) == ZT_OK)
      return ZT_OK;
    void *d_in;
    ZT_TRY(scratch(c, 0, n, &d_in));
    ZT_TRY(upload(c, d_in, in, n, c->stream));
    uint8_t *d_out = nullptr;
    size_t ol = 0, eip = 0;
    int seg = inflate_segments_dev(c, (const uint8_t *)d_in, n, index, &d_out, 0, &ol, &eip, c->stream);
    // no sync points: speculative parallel decode at arbitrary bit offsets
    if (seg >= 1) seg = inflate_general_dev(c, (const uint8_t *)d_in, n, index, &d_out, 0, &ol, &eip, c->stream);
    if (seg < 0) return seg;
    if (seg == 0) {
      uint8_t *h = host_out(ol, true);
      if (!h) return set_error(ZT_E_NOMEM, "host allocation failed");
      const int rc = download(c, h, d_out, ol, c->stream);
      if (rc) {
        zt_free(h);
        return rc;
      }
      *out = h;
      *out_len = ol;
      if (end_ip) *end_ip = eip;
      return ZT_OK;
    }
  }
  int st = 0;
  size_t ip = 0;
  const uint8_t *p = in;
  int rc = inflate_host_batch(&p, &n, &index, 1, opts, out, out_len, &ip, &st);
  if (end_ip) *end_ip = ip;
  return rc;
}

}  // extern "C"

// zt_inflate_raw_resume / _final: `final_input` = the caller has no more
// input, so every kernel status is the stream's own (running out is an error)
static int resume_impl(const uint8_t *in, size_t n, uint64_t bit_pos, const uint8_t *window, size_t wlen,
                       uint8_t **out, size_t *out_len, uint64_t *end_bits, int *finished, int final_input) {
  if (!out || !out_len || !end_bits || !finished) return set_error(ZT_E_ARG, "null output");
  if ((n && !in) || (wlen && !window)) return set_error(ZT_E_ARG, "null input");
  if (bit_pos > (uint64_t)n * 8) return set_error(ZT_E_ARG, "bit position past the end of the input");
  *out = nullptr;
  *out_len = 0;
  *end_bits = bit_pos;
  *finished = 0;
  if (wlen > 32768) {  // only the last 32 KiB can be referenced
    window += wlen - 32768;
    wlen = 32768;
  }
  // the decoder reads the caller's bytes from the byte holding bit_pos on
  // (byte alignment kept: stored blocks stay aligned), skips the bits of that
  // byte already used, and starts with the window in its history
  const size_t byte = (size_t)(bit_pos >> 3);
  const unsigned sh = (unsigned)(bit_pos & 7);
  const size_t m = n - byte;
  if ((uint64_t)m * 8 <= sh) return ZT_OK;  // nothing new to decode
  DeviceCtx *c;
  ZT_TRY(get_ctx(&c));
  std::lock_guard<std::recursive_mutex> ctx_lock(c->mu);
  void *d_in, *d_jobs;
  const size_t in_bytes = align_up(m, 256);
  ZT_TRY(scratch(c, 0, in_bytes + wlen + 16, &d_in));
  ZT_TRY(upload(c, d_in, in + byte, m, c->stream));
  const uint8_t *d_hist = (const uint8_t *)d_in + in_bytes;
  if (wlen) ZT_HIP(hipMemcpyAsync((void *)d_hist, window, wlen, hipMemcpyHostToDevice, c->stream));
  ZT_TRY(scratch(c, 2, sizeof(InfJob) + sizeof(InfResult) + 256, &d_jobs));
  InfResult *d_res = (InfResult *)((uint8_t *)d_jobs + align_up(sizeof(InfJob), 256));
  size_t cap = std::max<size_t>(65536, m * 4);
  for (int pass = 0; pass < 2; ++pass) {
    void *d_out;
    ZT_TRY(scratch(c, 1, cap, &d_out));
    InfJob j{};
    j.in = (const uint8_t *)d_in;
    j.n = m;
    j.out = (uint8_t *)d_out;
    j.cap = cap;
    j.resume = 1;
    j.start_bit = sh;
    j.hist = d_hist;
    j.hist_len = (uint32_t)wlen;
    InfResult r;
    ZT_HIP(hipMemcpyAsync(d_jobs, &j, sizeof j, hipMemcpyHostToDevice, c->stream));
    ZT_TRY(inflate_jobs_dev((const InfJob *)d_jobs, d_res, 1, c->stream));
    ZT_TRY(readback(c, &r, d_res, sizeof r, c->stream));
    // running out of input (the reader's end-of-input statuses, or any error
    // within the last 64 bits, where a peek may have seen the zeros past the
    // end) means "more input needed"; an error before that is the stream's own
    const bool truncated = !final_input && (r.status == ZT_E_INPUT_BROKEN || r.status == ZT_E_STORED_LEN ||
                                            r.status == ZT_E_STORED_NLEN || r.status == ZT_E_INVALID_CODE_LENGTH ||
                                            r.stop_bits + 64 > (uint64_t)m * 8);
    if (r.status != ZT_OK && !truncated) return inflate_error(r.status, r.detail);
    const uint64_t done = (r.status == ZT_OK ? r.out_len : r.blk_op) - wlen;  // new bytes
    if (done > cap) {  // decoded past the output guess: again with the exact size
      cap = (size_t)done;
      continue;
    }
    uint8_t *h = host_out(done);
    if (!h) return set_error(ZT_E_NOMEM, "host allocation failed");
    const int rc = download(c, h, d_out, done, c->stream);
    if (rc) {
      zt_free(h);
      return rc;
    }
    *out = h;
    *out_len = done;
    *end_bits = (uint64_t)byte * 8 + r.blk_bits;
    *finished = r.status == ZT_OK ? 1 : 0;
    return ZT_OK;
  }
  return set_error(ZT_E_INTERNAL, "resume: output size did not settle");
}

extern "C" {

int zt_inflate_raw_resume(const uint8_t *in, size_t n, uint64_t bit_pos, const uint8_t *window, size_t wlen,
                          uint8_t **out, size_t *out_len, uint64_t *end_bits, int *finished) {
  return resume_impl(in, n, bit_pos, window, wlen, out, out_len, end_bits, finished, 0);
}

int zt_inflate_raw_resume_final(const uint8_t *in, size_t n, uint64_t bit_pos, const uint8_t *window, size_t wlen,
                                uint8_t **out, size_t *out_len, uint64_t *end_bits, int *finished) {
  return resume_impl(in, n, bit_pos, window, wlen, out, out_len, end_bits, finished, 1);
}

int zt_inflate_raw_batch(const uint8_t *const *in, const size_t *n, size_t count, const zt_inflate_opts *opts,
                         uint8_t **out, size_t *out_len, size_t *end_ip, int *status) {
  if (count == 0) return ZT_OK;
  if (!in || !n || !out || !out_len || !status) return set_error(ZT_E_ARG, "null argument");
  return inflate_host_batch(in, n, nullptr, count, opts, out, out_len, end_ip, status);
}

}  // extern "C"
