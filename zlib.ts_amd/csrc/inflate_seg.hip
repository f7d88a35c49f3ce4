// inflate_seg.hip -- segment-parallel inflate of one large stream.
//
// Our deflate starts an independent segment every 1 MiB of input (no match
// reaches behind a segment start) and announces it with two empty stored
// blocks, 00 00 00 FF FF 00 00 00 FF FF (deflate.hip).  Any stream carrying
// that pattern is decoded here as follows:
//   1. find_restarts: every position is tested for the 10-byte pattern
//      (one 16-byte window per thread, HBM-bound), candidates are appended;
//   2. the candidates are sorted and every candidate is decoded as a segment
//      by its own wavefront (inflate.hip, InfJob::stops): a segment ends where
//      a stored block ends exactly on a later candidate;
//   3. the host follows the chain from the stream start (segment -> the
//      candidate it stopped on -> ...), so candidates that lie inside data are
//      never used.  A segment decoded on its own gives the stream's bytes iff
//      none of its matches reaches behind its start -- inflate.hip reports such
//      a match as "invalid distance" -- so any error on the chain falls back to
//      the one-wave decode, which also yields the reference's exact error;
//   4. the chain's outputs are compacted into the destination (64 KiB pieces).
// Reference behaviour replaced: src/RawInflate.ts:127-143 (decompress of one
// stream); results are identical to the sequential decode by construction.
#include <algorithm>
#include <vector>

#include "zt_internal.h"

namespace zt {

namespace {

constexpr uint32_t kMaxCand = 1u << 20;
constexpr uint64_t kPiece = 65536;

__global__ __launch_bounds__(256) void find_restarts(const uint8_t *__restrict__ in, uint64_t lo, uint64_t n,
                                                     uint64_t *__restrict__ list, uint32_t *__restrict__ count) {
  const uint64_t base = (lo & ~uint64_t(15)) + ((uint64_t)blockIdx.x * 256 + threadIdx.x) * 16;
  if (base >= n) return;
  uint8_t b[32];
#pragma unroll
  for (int j = 0; j < 32; ++j) b[j] = (base + j < n) ? in[base + j] : 1;
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const uint64_t p = base + j;
    if (b[j + 3] == 0xFF && b[j + 4] == 0xFF && b[j + 8] == 0xFF && b[j + 9] == 0xFF && b[j] == 0 &&
        b[j + 1] == 0 && b[j + 2] == 0 && b[j + 5] == 0 && b[j + 6] == 0 && b[j + 7] == 0 && p >= lo &&
        p + 10 <= n) {
      const uint32_t k = atomicAdd(count, 1u);
      if (k < kMaxCand) list[k] = p + 10;
    }
  }
}

struct Piece {
  const uint8_t *src;
  uint8_t *dst;
  uint64_t len;
};

__global__ __launch_bounds__(256) void copy_pieces(const Piece *__restrict__ pieces) {
  const Piece pc = pieces[blockIdx.x];
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  if (((reinterpret_cast<uintptr_t>(pc.src) | reinterpret_cast<uintptr_t>(pc.dst)) & 15) == 0) {
    const uint64_t nv = pc.len >> 4;
    const u32x4 *s = reinterpret_cast<const u32x4 *>(pc.src);
    u32x4 *d = reinterpret_cast<u32x4 *>(pc.dst);
    for (uint64_t i = threadIdx.x; i < nv; i += 256) d[i] = __builtin_nontemporal_load(&s[i]);
    for (uint64_t i = nv * 16 + threadIdx.x; i < pc.len; i += 256) pc.dst[i] = pc.src[i];
  } else {
    for (uint64_t i = threadIdx.x; i < pc.len; i += 256) pc.dst[i] = pc.src[i];
  }
}

size_t align256(size_t v) { return (v + 255) & ~size_t(255); }

}  // namespace

int inflate_segments_dev(DeviceCtx *c, const uint8_t *d_in, size_t n, size_t index, uint8_t **d_out_io,
                         size_t out_cap, size_t *out_len, size_t *end_ip, hipStream_t s) {
  if (n < index + (1u << 18)) return 1;  // small: one wave is as fast
  // 1. restart candidates
  void *d_cand;
  ZT_TRY(scratch(c, 5, 256 + (size_t)kMaxCand * 8, &d_cand));
  uint32_t *d_count = static_cast<uint32_t *>(d_cand);
  uint64_t *d_list = reinterpret_cast<uint64_t *>(static_cast<uint8_t *>(d_cand) + 256);
  ZT_HIP(hipMemsetAsync(d_count, 0, 4, s));
  const uint64_t span = n - (index & ~size_t(15));
  const uint32_t grid = (uint32_t)((span + 16 * 256 - 1) / (16 * 256));
  find_restarts<<<grid, 256, 0, s>>>(d_in, index, n, d_list, d_count);
  ZT_HIP(hipGetLastError());
  uint32_t cnt = 0;
  ZT_HIP(hipMemcpyAsync(&cnt, d_count, 4, hipMemcpyDeviceToHost, s));
  ZT_HIP(hipStreamSynchronize(s));
  if (cnt == 0 || cnt > kMaxCand) return 1;
  std::vector<uint64_t> cand(cnt);
  ZT_HIP(hipMemcpyAsync(cand.data(), d_list, (size_t)cnt * 8, hipMemcpyDeviceToHost, s));
  ZT_HIP(hipStreamSynchronize(s));
  std::sort(cand.begin(), cand.end());
  cand.erase(std::unique(cand.begin(), cand.end()), cand.end());
  cand.erase(std::remove_if(cand.begin(), cand.end(), [&](uint64_t p) { return p <= index || p >= n; }),
             cand.end());
  if (cand.empty()) return 1;
  // 2. one wave per segment (candidate), outputs into per-segment scratch
  const size_t units = cand.size() + 1;
  std::vector<uint64_t> start(units);
  start[0] = index;
  for (size_t i = 1; i < units; ++i) start[i] = cand[i - 1];
  std::vector<size_t> cap(units), off(units);
  size_t total_cap = 0;
  for (size_t i = 0; i < units; ++i) {
    const uint64_t e = i + 1 < units ? start[i + 1] : n;
    cap[i] = align256((e - start[i]) * 16 + 65536);
    off[i] = total_cap;
    total_cap += cap[i];
  }
  void *d_units, *d_meta;
  ZT_TRY(scratch(c, 4, total_cap, &d_units));
  const size_t stops_bytes = align256(cand.size() * 8);
  const size_t jobs_bytes = align256(units * sizeof(InfJob));
  ZT_TRY(scratch(c, 6, stops_bytes + jobs_bytes + align256(units * sizeof(InfResult)), &d_meta));
  uint64_t *d_stops = static_cast<uint64_t *>(d_meta);
  InfJob *d_jobs = reinterpret_cast<InfJob *>(static_cast<uint8_t *>(d_meta) + stops_bytes);
  InfResult *d_res = reinterpret_cast<InfResult *>(static_cast<uint8_t *>(d_meta) + stops_bytes + jobs_bytes);
  std::vector<InfJob> jobs(units);
  for (size_t i = 0; i < units; ++i) {
    InfJob &j = jobs[i];
    j = InfJob{};
    j.in = d_in;
    j.n = n;
    j.start = start[i];
    j.out = static_cast<uint8_t *>(d_units) + off[i];
    j.cap = cap[i];
    j.strict = 0;
    j.stops = d_stops;
    j.stop_first = (uint32_t)i;  // cand[i] is the next segment start
    j.stop_count = cand.size();
  }
  ZT_HIP(hipMemcpyAsync(d_stops, cand.data(), cand.size() * 8, hipMemcpyHostToDevice, s));
  ZT_HIP(hipMemcpyAsync(d_jobs, jobs.data(), units * sizeof(InfJob), hipMemcpyHostToDevice, s));
  ZT_TRY(timing_begin(c, s));
  ZT_TRY(inflate_jobs_dev(d_jobs, d_res, (int)units, s));
  ZT_TRY(timing_end(c, s));
  std::vector<InfResult> res(units);
  ZT_HIP(hipMemcpyAsync(res.data(), d_res, units * sizeof(InfResult), hipMemcpyDeviceToHost, s));
  ZT_HIP(hipStreamSynchronize(s));
  ZT_TRY(timing_collect(c, &c->times.inflate_ms, &c->times.inflate_launches));
  // 3. the chain from the stream start
  std::vector<size_t> chain;
  size_t u = 0;
  for (;;) {
    const InfResult &r = res[u];
    if (r.status != ZT_OK) return 1;  // exact error (or a match behind a false start): one wave decides
    chain.push_back(u);
    if (r.stop_idx < 0) break;
    const size_t nx = (size_t)r.stop_idx + 1;
    if (nx <= u || nx >= units) return 1;
    u = nx;
  }
  // segments that outgrew their scratch: decode again with the exact size
  std::vector<size_t> redo;
  for (size_t k : chain)
    if (res[k].out_len > cap[k]) redo.push_back(k);
  std::vector<const uint8_t *> src(units, nullptr);
  for (size_t k : chain) src[k] = static_cast<const uint8_t *>(d_units) + off[k];
  if (!redo.empty()) {
    size_t tot = 0;
    std::vector<size_t> roff(redo.size());
    for (size_t i = 0; i < redo.size(); ++i) {
      roff[i] = tot;
      tot += align256(res[redo[i]].out_len);
    }
    void *d_redo;
    ZT_TRY(scratch(c, 7, tot, &d_redo));
    std::vector<InfJob> rj(redo.size());
    for (size_t i = 0; i < redo.size(); ++i) {
      rj[i] = jobs[redo[i]];
      rj[i].out = static_cast<uint8_t *>(d_redo) + roff[i];
      rj[i].cap = res[redo[i]].out_len;
      src[redo[i]] = rj[i].out;
    }
    ZT_HIP(hipMemcpyAsync(d_jobs, rj.data(), rj.size() * sizeof(InfJob), hipMemcpyHostToDevice, s));
    ZT_TRY(inflate_jobs_dev(d_jobs, d_res, (int)rj.size(), s));
    std::vector<InfResult> rr(redo.size());
    ZT_HIP(hipMemcpyAsync(rr.data(), d_res, rr.size() * sizeof(InfResult), hipMemcpyDeviceToHost, s));
    ZT_HIP(hipStreamSynchronize(s));
    for (size_t i = 0; i < redo.size(); ++i)
      if (rr[i].status != ZT_OK || rr[i].out_len != res[redo[i]].out_len) return 1;
  }
  // 4. compaction
  size_t total = 0;
  for (size_t k : chain) total += res[k].out_len;
  *out_len = total;
  *end_ip = res[chain.back()].end_ip;
  uint8_t *d_out = *d_out_io;
  if (!d_out) {  // caller wants a library-owned buffer (scratch slot 1)
    void *p;
    ZT_TRY(scratch(c, 1, total ? total : 1, &p));
    d_out = static_cast<uint8_t *>(p);
    *d_out_io = d_out;
  } else if (total > out_cap) {
    return set_error(ZT_E_ARG, "output capacity too small");
  }
  std::vector<Piece> pieces;
  size_t pos = 0;
  for (size_t k : chain) {
    const size_t len = res[k].out_len;
    for (size_t a = 0; a < len; a += kPiece)
      pieces.push_back(Piece{src[k] + a, d_out + pos + a, std::min<uint64_t>(kPiece, len - a)});
    pos += len;
  }
  if (!pieces.empty()) {
    void *d_pieces;
    ZT_TRY(scratch(c, 2, pieces.size() * sizeof(Piece), &d_pieces));
    ZT_HIP(hipMemcpyAsync(d_pieces, pieces.data(), pieces.size() * sizeof(Piece), hipMemcpyHostToDevice, s));
    copy_pieces<<<(unsigned)pieces.size(), 256, 0, s>>>(static_cast<const Piece *>(d_pieces));
    ZT_HIP(hipGetLastError());
  }
  ZT_HIP(hipStreamSynchronize(s));
  return ZT_OK;
}

}  // namespace zt
