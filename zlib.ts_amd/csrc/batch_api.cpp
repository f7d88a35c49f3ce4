// batch_api.cpp -- many independent buffers per call (configs C4 and C2's
// producer side; include/zt.h): zt_gzip_compress_batch, zt_zlib_compress_batch
// and zt_deflate_raw_batch.
//
// Per device, one pipeline for the whole share: the buffers are packed into
// pinned staging at 32 KiB boundaries and uploaded with one copy; the batch
// deflate pipeline (deflate.hip, one match workgroup per block so no history
// crosses buffers) runs on the main stream while the batched CRC-32 /
// Adler-32 kernels read the same device bytes on the second stream; one copy
// brings every stream back.  With zt_set_devices(mask) the buffers are split
// over the devices by longest-processing-time (largest first onto the least
// loaded device) and each device's share runs on its own host thread.
// Replaces a loop of new GZip(input).compress() (src/GZip.ts:96-194),
// new Deflate(input).compress() (src/Deflate.ts:60-99) and
// new RawDeflate(input).compress() (src/RawDeflate.ts:87-114).
#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "zt_internal.h"

namespace zt {

namespace {

constexpr uint64_t kBlk = 32768;

// ZT_BATCH_STAGES=1: host-only stage timers of one device's share (JSON line
// on stderr per share) -- packing into pinned staging and framing the members
// are the host work that has to keep up with k devices on a node
// (tools/c4_host_stages.py).  Measurement only.
double stage_now() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
bool stages_on() {
  static const bool on = getenv("ZT_BATCH_STAGES") != nullptr;
  return on;
}
struct StageTimes {
  double pack_ms = 0, frame_ms = 0, wall_ms = 0;
  uint64_t in_bytes = 0, out_bytes = 0;
  size_t items = 0, groups = 0;
  void report(int dev) const {
    if (!stages_on()) return;
    fprintf(stderr,
            "{\"zt_batch_stages\": 1, \"device\": %d, \"items\": %zu, \"groups\": %zu, \"in_bytes\": %llu, "
            "\"out_bytes\": %llu, \"pack_ms\": %.3f, \"frame_ms\": %.3f, \"wall_ms\": %.3f}\n",
            dev, items, groups, (unsigned long long)in_bytes, (unsigned long long)out_bytes, pack_ms, frame_ms,
            wall_ms);
  }
};

size_t round_blk(size_t n) { return (n + kBlk - 1) / kBlk * kBlk; }

// fills out[i] (malloc'd: prefix | stream | trailer) for item i
struct Framing {
  enum Kind { RAW, GZIP, ZLIB } kind;
  std::vector<uint8_t> prefix;
  size_t trailer;
};

// (dst: the item's place in a batch slab, or null for its own allocation)
int frame_item(const Framing &fr, size_t n_in, const uint8_t *body, size_t blen, uint32_t crc, uint32_t adler,
               uint8_t **out, size_t *out_len, uint8_t *dst = nullptr) {
  const size_t total = fr.prefix.size() + blen + fr.trailer;
  uint8_t *h = dst ? dst : host_out(total);
  if (!h) return set_error(ZT_E_NOMEM, "host allocation failed");
  if (!fr.prefix.empty()) memcpy(h, fr.prefix.data(), fr.prefix.size());
  if (blen) memcpy(h + fr.prefix.size(), body, blen);
  uint8_t *t = h + fr.prefix.size() + blen;
  if (fr.kind == Framing::GZIP) {  // CRC-32, ISIZE (src/GZip.ts:179-185)
    for (int k = 0; k < 4; ++k) t[k] = (crc >> (8 * k)) & 0xFF;
    for (int k = 0; k < 4; ++k) t[4 + k] = ((uint32_t)n_in >> (8 * k)) & 0xFF;
  } else if (fr.kind == Framing::ZLIB) {  // Adler-32 big-endian (src/Deflate.ts:95)
    for (int k = 0; k < 4; ++k) t[k] = (adler >> (24 - 8 * k)) & 0xFF;
  }
  *out = h;
  *out_len = total;
  return ZT_OK;
}

// items [k0, k0 + nb) framed into one slab (slab_out): their offsets, and
// the slab (null when it cannot be allocated)
uint8_t *frame_slab(const Framing &fr, const uint64_t *oo, size_t nb, std::vector<size_t> &soff) {
  soff.resize(nb);
  size_t tot = 0;
  for (size_t j = 0; j < nb; ++j) {
    soff[j] = tot;
    tot += (fr.prefix.size() + (oo[j + 1] - oo[j]) + fr.trailer + 64) & ~size_t(63);
  }
  return slab_out(tot, nb);
}

// Large shares (>= kGroupMin padded bytes): the items are cut, in order, into
// groups of about 1/6 of the share (>= 128 MiB) and run as a three-stage
// pipeline, so PCIe and the host work overlap the GPU: group g + 1 is packed
// into pinned staging and uploaded (stream c->up, one host thread) while
// group g is checksummed (c->aux) and deflated (c->stream, the caller's
// thread) and group g - 1 comes back and is framed into the members (stream
// c->dn, one host thread).  Groups are independent batch pipelines (no item
// spans two), so every member is the one the single pipeline writes.
constexpr uint64_t kGroupMin = 256ull << 20;

int batch_grouped(DeviceCtx *c, const uint8_t *const *in, const std::vector<size_t> &work,
                  const std::vector<uint64_t> &off, const std::vector<uint64_t> &len, uint64_t padded, int ct, int lv,
                  const Framing &fr, uint8_t **out, size_t *out_len, StageTimes &tm) {
  const size_t m = work.size();
  const bool sums = fr.kind != Framing::RAW;
  // groups [gk[g], gk[g + 1]) of items
  // tuning hook: ZT_BATCH_GROUPS = groups per share (default 6)
  static const int ng_env = getenv("ZT_BATCH_GROUPS") ? atoi(getenv("ZT_BATCH_GROUPS")) : 0;
  const uint64_t target = std::max<uint64_t>(padded / (ng_env > 0 ? ng_env : 6), 64ull << 20);
  std::vector<size_t> gk{0};
  for (size_t k = 0; k < m; ++k)
    if (k + 1 < m && off[k + 1] - off[gk.back()] >= target) gk.push_back(k + 1);
  gk.push_back(m);
  const size_t ng = gk.size() - 1;
  auto gbeg = [&](size_t g) { return off[gk[g]]; };
  auto gend = [&](size_t g) { return gk[g + 1] < m ? off[gk[g + 1]] : padded; };
  auto obound = [](uint64_t p) { return (p + p / 8 + 1024 * (p / kBlk + 1) + 4096 + 255) & ~uint64_t(255); };
  uint64_t gmax = 0, obmax = 0, obsum = 0;
  std::vector<uint64_t> ooff(ng + 1, 0);  // device output region of group g
  for (size_t g = 0; g < ng; ++g) {
    gmax = std::max(gmax, gend(g) - gbeg(g));
    obmax = std::max(obmax, obound(gend(g) - gbeg(g)));
    ooff[g + 1] = ooff[g] + obound(gend(g) - gbeg(g));
  }
  obsum = ooff[ng];
  void *d_in, *d_out, *d_scr, *d_sums = nullptr, *p;
  ZT_TRY(scratch(c, 0, padded + 64, &d_in));
  ZT_TRY(scratch(c, 1, obsum, &d_out));
  const size_t ss = deflate_batch_scratch_bytes(c, gmax);
  ZT_TRY(scratch(c, 3, ss, &d_scr));
  if (sums) ZT_TRY(scratch(c, 18, 8 * m, &d_sums));
  uint8_t *stage_in[2], *stage_out;
  ZT_TRY(pinned(c, gmax, &p, 0));
  stage_in[0] = static_cast<uint8_t *>(p);
  ZT_TRY(pinned(c, gmax, &p, 6));
  stage_in[1] = static_cast<uint8_t *>(p);
  ZT_TRY(pinned(c, obmax, &p, 7));
  stage_out = static_cast<uint8_t *>(p);
  if (!c->up) ZT_HIP(hipStreamCreateWithFlags(&c->up, hipStreamNonBlocking));
  if (!c->dn) ZT_HIP(hipStreamCreateWithFlags(&c->dn, hipStreamNonBlocking));
  std::vector<hipEvent_t> landed(ng, nullptr), staged(2, nullptr);
  struct EvFree {
    std::vector<hipEvent_t> &a, &b;
    ~EvFree() {
      for (auto e : a)
        if (e) (void)hipEventDestroy(e);
      for (auto e : b)
        if (e) (void)hipEventDestroy(e);
    }
  } ev_free{landed, staged};
  for (auto &e : landed) ZT_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  for (auto &e : staged) ZT_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));

  std::vector<uint32_t> hsums(2 * m, 0);
  std::vector<uint64_t> oo(m + ng, 0);  // group g's stream offsets at oo[gk[g] + g ..]
  std::mutex mu;
  std::condition_variable cv;
  size_t uploaded = 0, computed = 0;
  int err = 0;
  std::string err_msg;
  auto fail = [&](int rc) {
    std::lock_guard<std::mutex> lk(mu);
    if (!err) {
      err = rc;
      err_msg = zt_last_error_message();
    }
    cv.notify_all();
  };
  auto wait_for = [&](const size_t &counter, size_t g) {
    std::unique_lock<std::mutex> lk(mu);
    cv.wait(lk, [&] { return counter > g || err; });
    return err == 0;
  };
  const int dev = c->phys;
  auto up_stage = [&]() -> int {
    ZT_HIP(hipSetDevice(dev));
    for (size_t g = 0; g < ng; ++g) {
      {
        std::lock_guard<std::mutex> lk(mu);
        if (err) return ZT_OK;
      }
      uint8_t *st = stage_in[g & 1];
      if (g >= 2) ZT_HIP(hipEventSynchronize(staged[g & 1]));  // its previous upload has left
      const uint64_t b = gbeg(g), nb = gk[g + 1] - gk[g];
      const double t0 = stage_now();
      parallel_copy(nb, [&](size_t j) {
        const size_t k = gk[g] + j;
        copy_to_staging(st + off[k] - b, in[work[k]], len[k]);
        memset(st + off[k] - b + len[k], 0, round_blk(len[k]) - len[k]);
      }, gend(g) - b);
      tm.pack_ms += stage_now() - t0;  // (this thread only)
      ZT_HIP(hipMemcpyAsync((uint8_t *)d_in + b, st, gend(g) - b, hipMemcpyHostToDevice, c->up));
      ZT_HIP(hipEventRecord(staged[g & 1], c->up));
      ZT_HIP(hipEventRecord(landed[g], c->up));
      std::lock_guard<std::mutex> lk(mu);
      uploaded = g + 1;
      cv.notify_all();
    }
    ZT_HIP(hipStreamSynchronize(c->up));
    return ZT_OK;
  };
  auto dn_stage = [&]() -> int {
    ZT_HIP(hipSetDevice(dev));
    for (size_t g = 0; g < ng; ++g) {
      if (!wait_for(computed, g)) return ZT_OK;
      const size_t k0 = gk[g], nb = gk[g + 1] - k0;
      const uint64_t *go = &oo[k0 + g];
      ZT_HIP(hipMemcpyAsync(stage_out, (uint8_t *)d_out + ooff[g], go[nb], hipMemcpyDeviceToHost, c->dn));
      ZT_HIP(hipStreamSynchronize(c->dn));
      std::vector<int> rcs(nb, ZT_OK);
      std::vector<size_t> soff;
      const double t0 = stage_now();
      uint8_t *slab = frame_slab(fr, go, nb, soff);
      if (!slab) return set_error(ZT_E_NOMEM, "host allocation failed");
      parallel_copy(nb, [&](size_t j) {
        const size_t k = k0 + j, i = work[k];
        rcs[j] = frame_item(fr, len[k], stage_out + go[j], go[j + 1] - go[j], hsums[2 * k], hsums[2 * k + 1], &out[i],
                            &out_len[i], slab + soff[j]);
      }, go[nb]);
      tm.frame_ms += stage_now() - t0;  // (this thread only)
      tm.out_bytes += go[nb];
      for (int rc : rcs)
        if (rc) return rc;
    }
    return ZT_OK;
  };
  std::thread tu([&] {
    if (int rc = up_stage()) fail(rc);
  });
  std::thread td([&] {
    if (int rc = dn_stage()) fail(rc);
  });
  for (size_t g = 0; g < ng; ++g) {
    if (!wait_for(uploaded, g)) break;
    const size_t k0 = gk[g], nb = gk[g + 1] - k0;
    const uint64_t b = gbeg(g);
    std::vector<uint64_t> ro(nb), rl(len.begin() + k0, len.begin() + k0 + nb);
    for (size_t j = 0; j < nb; ++j) ro[j] = off[k0 + j] - b;
    auto step = [&]() -> int {
      ZT_HIP(hipStreamWaitEvent(c->stream, landed[g], 0));
      if (sums) {
        ZT_HIP(hipStreamWaitEvent(c->aux, landed[g], 0));
        ZT_TRY(checksums_batch_dev(c, (const uint8_t *)d_in + b, nb, ro.data(), rl.data(),
                                   (uint32_t *)d_sums + 2 * k0, c->aux));
        ZT_HIP(hipMemcpyAsync(hsums.data() + 2 * k0, (uint32_t *)d_sums + 2 * k0, 8 * nb, hipMemcpyDeviceToHost,
                              c->aux));
      }
      ZT_TRY(deflate_batch_dev_run(c, (const uint8_t *)d_in + b, nb, ro.data(), rl.data(), ct, lv,
                                   (uint8_t *)d_out + ooff[g], &oo[k0 + g], d_scr, ss, c->stream));
      if (sums) ZT_HIP(hipStreamSynchronize(c->aux));
      return ZT_OK;
    };
    if (int rc = step()) {
      fail(rc);
      break;
    }
    std::lock_guard<std::mutex> lk(mu);
    computed = g + 1;
    cv.notify_all();
  }
  tu.join();
  td.join();
  tm.groups = ng;
  if (err) return set_error(err, err_msg);
  return ZT_OK;
}

// one device's share: items `ids` of the batch
int batch_on_device(int dev, const uint8_t *const *in, const size_t *n, const std::vector<size_t> &ids, int ct,
                    int lv, const Framing &fr, uint8_t **out, size_t *out_len, std::string *err) {
  auto fail = [&](int rc) {
    *err = zt_last_error_message();
    return rc;
  };
  if (zt_set_device(dev)) return fail(ZT_E_NO_DEVICE);
  DeviceCtx *c;
  if (int rc = get_ctx(&c)) return fail(rc);
  std::lock_guard<std::recursive_mutex> ctx_lock(c->mu);
  const bool sums = fr.kind != Framing::RAW;
  // empty inputs: a final empty stored block, as the one-buffer calls write
  // (deflate.hip) -- no device work
  std::vector<size_t> work;
  for (size_t i : ids) {
    if (n[i] == 0) {
      static const uint8_t empty_stored[5] = {0x01, 0x00, 0x00, 0xFF, 0xFF};
      const int rc = frame_item(fr, 0, empty_stored, 5, 0, 1, &out[i], &out_len[i]);
      if (rc) return fail(rc);
    } else {
      work.push_back(i);
    }
  }
  if (work.empty()) return ZT_OK;
  const size_t m = work.size();
  std::vector<uint64_t> off(m), len(m);
  uint64_t padded = 0, in_bytes = 0;
  for (size_t k = 0; k < m; ++k) {
    off[k] = padded;
    len[k] = n[work[k]];
    padded += round_blk(len[k]);
    in_bytes += len[k];
  }
  StageTimes tm;
  tm.items = m;
  tm.in_bytes = in_bytes;
  const double t_start = stage_now();
  struct Report {
    StageTimes &tm;
    double t0;
    int dev;
    ~Report() {
      tm.wall_ms = stage_now() - t0;
      tm.report(dev);
    }
  } report{tm, t_start, dev};
  if (ct != 0 && padded >= kGroupMin && m >= 2) {
    const int rc = batch_grouped(c, in, work, off, len, padded, ct, lv, fr, out, out_len, tm);
    return rc ? fail(rc) : ZT_OK;
  }
  void *d_in, *h_stage;
  if (int rc = scratch(c, 0, padded + 64, &d_in)) return fail(rc);
  if (int rc = pinned(c, padded, &h_stage, 0)) return fail(rc);
  uint8_t *stage = static_cast<uint8_t *>(h_stage);
  const double t_pack = stage_now();
  parallel_copy(m, [&](size_t k) {
    copy_to_staging(stage + off[k], in[work[k]], len[k]);
    memset(stage + off[k] + len[k], 0, round_blk(len[k]) - len[k]);
  }, in_bytes);
  tm.pack_ms += stage_now() - t_pack;
  tm.groups = 1;
  ZT_HIP(hipMemcpyAsync(d_in, stage, padded, hipMemcpyHostToDevice, c->stream));
  // checksums on the second stream, over the same device bytes
  std::vector<uint32_t> hsums(2 * m, 0);
  void *d_sums = nullptr;
  struct AuxWait {
    hipStream_t s;
    ~AuxWait() { (void)hipStreamSynchronize(s); }
  } aux_wait{c->aux};
  if (sums) {
    if (int rc = scratch(c, 18, 8 * m, &d_sums)) return fail(rc);
    ZT_HIP(hipEventRecord(c->aux_ev, c->stream));
    ZT_HIP(hipStreamWaitEvent(c->aux, c->aux_ev, 0));
    if (int rc = checksums_batch_dev(c, (const uint8_t *)d_in, m, off.data(), len.data(), (uint32_t *)d_sums, c->aux))
      return fail(rc);
    ZT_HIP(hipMemcpyAsync(hsums.data(), d_sums, 8 * m, hipMemcpyDeviceToHost, c->aux));
  }
  std::vector<uint64_t> oo(m + 1, 0);
  uint8_t *body_host = nullptr;
  std::vector<uint8_t> stored_host;
  if (ct == 0) {
    // stored blocks of <= 65535 bytes (src/RawDeflate.ts:93-100,122-153): framing only
    uint64_t tot = 0;
    for (size_t k = 0; k < m; ++k) {
      oo[k] = tot;
      tot += len[k] + 5 * ((len[k] + 65534) / 65535);
    }
    oo[m] = tot;
    stored_host.resize(tot);
    for (size_t k = 0; k < m; ++k) {
      uint8_t *o = stored_host.data() + oo[k];
      const uint8_t *src = in[work[k]];
      for (uint64_t p = 0; p < len[k]; p += 65535) {
        const uint32_t l = (uint32_t)std::min<uint64_t>(65535, len[k] - p);
        o[0] = p + l == len[k] ? 1 : 0;
        o[1] = l & 0xFF;
        o[2] = l >> 8;
        o[3] = ~l & 0xFF;
        o[4] = (~l >> 8) & 0xFF;
        memcpy(o + 5, src + p, l);
        o += 5 + l;
      }
    }
    body_host = stored_host.data();
  } else {
    const size_t ob = padded + padded / 8 + 1024 * (padded / kBlk + 1) + 4096;
    void *d_out, *d_scr;
    if (int rc = scratch(c, 1, ob, &d_out)) return fail(rc);
    const size_t ss = deflate_batch_scratch_bytes(c, padded);
    if (int rc = scratch(c, 3, ss, &d_scr)) return fail(rc);
    if (int rc = deflate_batch_dev_run(c, (const uint8_t *)d_in, m, off.data(), len.data(), ct, lv,
                                       (uint8_t *)d_out, oo.data(), d_scr, ss, c->stream))
      return fail(rc);
    // The members are framed on the device (prefix | stream | trailer, at
    // their slab offsets) and come back with one copy -- straight into the
    // slab when it is a registered pool buffer (a caller batching again after
    // freeing the last outputs): the host only lays the slab out.  Host
    // framing (the slab filled from a staged copy of the streams) was a
    // quarter of a device thread's host time on a node's worth of devices
    // (tools/c4_host_stages.py).
    const double t_frame = stage_now();
    const uint32_t plen = (uint32_t)fr.prefix.size(), tl = (uint32_t)fr.trailer;
    std::vector<FrameItem> fi(m);
    std::vector<size_t> soff(m);
    size_t tot = 0;
    for (size_t k = 0; k < m; ++k) {
      soff[k] = tot;
      fi[k] = FrameItem{oo[k], tot, (uint32_t)(oo[k + 1] - oo[k]), (uint32_t)len[k]};
      tot += (plen + (oo[k + 1] - oo[k]) + tl + 64) & ~size_t(63);
    }
    const size_t fr_bytes = (tot + 255) & ~size_t(255), it_bytes = (m * sizeof(FrameItem) + 255) & ~size_t(255);
    void *d_fr;
    if (int rc = scratch(c, 27, fr_bytes + it_bytes + plen + 256, &d_fr)) return fail(rc);
    uint8_t *d_framed = static_cast<uint8_t *>(d_fr);
    FrameItem *d_items = reinterpret_cast<FrameItem *>(d_framed + fr_bytes);
    uint8_t *d_prefix = d_framed + fr_bytes + it_bytes;
    ZT_HIP(hipMemcpyAsync(d_items, fi.data(), m * sizeof(FrameItem), hipMemcpyHostToDevice, c->stream));
    if (plen) ZT_HIP(hipMemcpyAsync(d_prefix, fr.prefix.data(), plen, hipMemcpyHostToDevice, c->stream));
    if (sums) {  // (the trailers need the checksums from the second stream)
      ZT_HIP(hipEventRecord(c->aux_ev, c->aux));
      ZT_HIP(hipStreamWaitEvent(c->stream, c->aux_ev, 0));
    }
    if (int rc = frame_members_dev(d_items, (uint32_t)m, d_prefix, plen,
                                   fr.kind == Framing::GZIP ? 8u : fr.kind == Framing::ZLIB ? 4u : 0u,
                                   static_cast<const uint8_t *>(d_out), static_cast<const uint32_t *>(d_sums),
                                   d_framed, c->stream))
      return fail(rc);
    uint8_t *slab = slab_out(tot, m, true);
    if (!slab) return fail(set_error(ZT_E_NOMEM, "host allocation failed"));
    const bool direct = host_direct(slab, tot);
    tm.frame_ms += stage_now() - t_frame;
    if (direct) {  // (DMA time, not host work: like the upload, outside the stage timers)
      ZT_HIP(hipMemcpyAsync(slab, d_framed, tot, hipMemcpyDeviceToHost, c->stream));
      ZT_HIP(hipStreamSynchronize(c->stream));
    } else {
      const double t_dl = stage_now();
      if (int rc = download(c, slab, d_framed, tot, c->stream)) return fail(rc);
      tm.frame_ms += stage_now() - t_dl;  // (staged: host copies)
    }
    ZT_HIP(hipStreamSynchronize(c->aux));
    for (size_t k = 0; k < m; ++k) {
      out[work[k]] = slab + soff[k];
      out_len[work[k]] = plen + (oo[k + 1] - oo[k]) + tl;
    }
    tm.out_bytes += oo[m];
    return ZT_OK;
  }
  ZT_HIP(hipStreamSynchronize(c->aux));
  int first_rc = ZT_OK;
  std::vector<int> rcs(m, ZT_OK);
  std::vector<size_t> soff;
  const double t_frame = stage_now();
  uint8_t *slab = frame_slab(fr, oo.data(), m, soff);
  if (!slab) return fail(set_error(ZT_E_NOMEM, "host allocation failed"));
  parallel_copy(m, [&](size_t k) {
    const size_t i = work[k];
    rcs[k] = frame_item(fr, len[k], body_host + oo[k], oo[k + 1] - oo[k], hsums[2 * k], hsums[2 * k + 1], &out[i],
                        &out_len[i], slab + soff[k]);
  }, oo[m]);
  tm.frame_ms += stage_now() - t_frame;
  tm.out_bytes += oo[m];
  for (int rc : rcs)
    if (rc && !first_rc) first_rc = rc;
  return first_rc ? fail(first_rc) : ZT_OK;
}

// split over the batch devices (LPT) and run every share on its own thread
int run_batch(const uint8_t *const *in, const size_t *n, size_t count, int ct, int lv, const Framing &fr,
              uint8_t **out, size_t *out_len, int *status) {
  for (size_t i = 0; i < count; ++i) {
    out[i] = nullptr;
    out_len[i] = 0;
    if (n[i] && !in[i]) return set_error(ZT_E_ARG, "null input");
  }
  const std::vector<int> devs = batch_devices();
  const size_t nd = devs.size();
  std::vector<std::vector<size_t>> share(nd);
  if (nd == 1) {
    share[0].resize(count);
    for (size_t i = 0; i < count; ++i) share[0][i] = i;
  } else {
    std::vector<size_t> order(count);
    for (size_t i = 0; i < count; ++i) order[i] = i;
    std::stable_sort(order.begin(), order.end(), [&](size_t a, size_t b) { return n[a] > n[b]; });
    std::vector<uint64_t> load(nd, 0);
    for (size_t i : order) {
      const size_t d = (size_t)(std::min_element(load.begin(), load.end()) - load.begin());
      share[d].push_back(i);
      load[d] += n[i] + 4096;  // + per-item cost
    }
    for (auto &v : share) std::sort(v.begin(), v.end());
  }
  std::vector<int> rc(nd, ZT_OK);
  std::vector<std::string> err(nd);
  const int caller_dev = current_device();
  if (nd == 1) {
    rc[0] = batch_on_device(devs[0], in, n, share[0], ct, lv, fr, out, out_len, &err[0]);
    zt_set_device(caller_dev);
  } else {
    std::vector<std::thread> th;
    for (size_t d = 0; d < nd; ++d)
      th.emplace_back([&, d] {
        // the host's copy threads split between the device threads (8 per
        // device thread put 64 on one GPU's 16-thread CPU share with 8
        // devices; 32 in all packed fastest: slowest device's host stages
        // 10.9 GiB/s with 16, 13.3 with 32, gpurun_out/r06ab);
        // ZT_BATCH_COPY_THREADS overrides the total
        static const size_t total = getenv("ZT_BATCH_COPY_THREADS") ? (size_t)atoi(getenv("ZT_BATCH_COPY_THREADS")) : 32;
        set_copy_threads(std::max<size_t>(2, total / nd));
        rc[d] = batch_on_device(devs[d], in, n, share[d], ct, lv, fr, out, out_len, &err[d]);
      });
    for (auto &t : th) t.join();
  }
  int first = ZT_OK;
  for (size_t d = 0; d < nd; ++d) {
    for (size_t i : share[d]) status[i] = rc[d];
    if (rc[d] && first == ZT_OK) {
      first = rc[d];
      set_error(rc[d], err[d]);
    }
  }
  if (first) {
    for (size_t i = 0; i < count; ++i) {
      zt_free(out[i]);
      out[i] = nullptr;
      out_len[i] = 0;
    }
  }
  return first;
}

int resolve_opts(const zt_deflate_opts *o, int *ct, int *lv) {
  int c = o ? o->compression_type : 2;
  int l = o ? o->level : -1;
  if (c < 0 || c > 2) return set_error(ZT_E_INVALID_COMPRESSION_TYPE, "invalid compression type");
  if (l < 0 || l > 9) l = 6;
  if (l == 0) c = 0;
  if (o && o->lazy > 0 && l < 4) l = 4;
  *ct = c;
  *lv = l;
  return ZT_OK;
}

}  // namespace
}  // namespace zt

using namespace zt;

extern "C" {

int zt_deflate_raw_batch(const uint8_t *const *in, const size_t *n, size_t count, const zt_deflate_opts *opts,
                         uint8_t **out, size_t *out_len, int *status) {
  if (count == 0) return ZT_OK;
  if (!in || !n || !out || !out_len || !status) return set_error(ZT_E_ARG, "null argument");
  int ct, lv;
  ZT_TRY(resolve_opts(opts, &ct, &lv));
  Framing fr{Framing::RAW, {}, 0};
  return run_batch(in, n, count, ct, lv, fr, out, out_len, status);
}

int zt_gzip_compress_batch(const uint8_t *const *in, const size_t *n, size_t count, const zt_gzip_opts *opts,
                           uint8_t **out, size_t *out_len, int *status) {
  if (count == 0) return ZT_OK;
  if (!in || !n || !out || !out_len || !status) return set_error(ZT_E_ARG, "null argument");
  int ct, lv;
  ZT_TRY(resolve_opts(opts ? &opts->deflate : nullptr, &ct, &lv));
  Framing fr{Framing::GZIP, {}, 8};
  gzip_header(opts, fr.prefix);
  return run_batch(in, n, count, ct, lv, fr, out, out_len, status);
}

int zt_crc32_batch(const uint8_t *const *in, const size_t *n, size_t count, uint32_t *crc_out) {
  if (count == 0) return ZT_OK;
  if (!in || !n || !crc_out) return set_error(ZT_E_ARG, "null argument");
  DeviceCtx *c;
  ZT_TRY(get_ctx(&c));
  std::lock_guard<std::recursive_mutex> ctx_lock(c->mu);
  std::vector<uint64_t> off(count), len(count);
  uint64_t tot = 0;
  for (size_t i = 0; i < count; ++i) {
    if (n[i] && !in[i]) return set_error(ZT_E_ARG, "null input");
    off[i] = tot;
    len[i] = n[i];
    tot += (n[i] + 255) & ~uint64_t(255);
  }
  void *d_in, *h, *d_sums;
  ZT_TRY(scratch(c, 0, tot + 64, &d_in));
  ZT_TRY(pinned(c, tot + 64, &h, 0));
  uint8_t *stage = static_cast<uint8_t *>(h);
  parallel_copy(count, [&](size_t i) { copy_to_staging(stage + off[i], in[i], n[i]); }, tot);
  ZT_HIP(hipMemcpyAsync(d_in, stage, tot ? tot : 1, hipMemcpyHostToDevice, c->stream));
  ZT_TRY(scratch(c, 18, 8 * count, &d_sums));
  ZT_TRY(checksums_batch_dev(c, (const uint8_t *)d_in, count, off.data(), len.data(), (uint32_t *)d_sums, c->stream));
  std::vector<uint32_t> sums(2 * count);
  ZT_HIP(hipMemcpyAsync(sums.data(), d_sums, 8 * count, hipMemcpyDeviceToHost, c->stream));
  ZT_HIP(hipStreamSynchronize(c->stream));
  for (size_t i = 0; i < count; ++i) crc_out[i] = sums[2 * i];
  return ZT_OK;
}

int zt_zlib_compress_batch(const uint8_t *const *in, const size_t *n, size_t count, const zt_deflate_opts *opts,
                           uint8_t **out, size_t *out_len, int *status) {
  if (count == 0) return ZT_OK;
  if (!in || !n || !out || !out_len || !status) return set_error(ZT_E_ARG, "null argument");
  int ct, lv;
  ZT_TRY(resolve_opts(opts, &ct, &lv));
  const uint32_t cmf = 0x78, flg0 = (uint32_t)(opts ? opts->compression_type : 2) << 6;
  Framing fr{Framing::ZLIB, {(uint8_t)cmf, (uint8_t)(flg0 | (31 - ((cmf << 8) + flg0) % 31))}, 4};
  return run_batch(in, n, count, ct, lv, fr, out, out_len, status);
}

}  // extern "C"
