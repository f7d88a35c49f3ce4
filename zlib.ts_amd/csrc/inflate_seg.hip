// inflate_seg.hip -- parallel inflate of one large stream (host orchestration).
//
// This engine's deflate ends every 32 KiB block on a byte-aligned empty stored
// block (00 00 FF FF: a *sync point* after it) and starts an independent
// 1 MiB segment with two more (the 10-byte restart marker
// 00 00 00 FF FF 00 00 00 FF FF; no match reaches behind it).  Streams that
// carry sync points are decoded in two phases (inflate_tok.hip):
//   1. find_syncs: every byte position is tested for the pattern (one 16-byte
//      window per thread, HBM-bound); sync points are appended, flagged when
//      the full restart marker precedes them;
//   2. tokenize_kernel: one wave per unit (stream start, or a sync point)
//      decodes blocks to tokens until it reaches another sync point;
//      (the candidate list is sorted and deduplicated, and the units' jobs
//      written, on the device: rocPRIM radix sort + scans; each unit's token
//      slot is bounded by the input bits up to the next candidate);
//   3. the host follows the chain from the stream start (unit -> the sync
//      point it stopped on -> the unit starting there ...), so sync points
//      that lie inside data are never used, and cuts the chain into segments
//      at restart markers; output offsets are the prefix sums of the units'
//      output lengths;
//   4. resolve_kernel: one wave per segment writes the bytes to their final
//      place.
// Any error on the chain, a unit that outgrew its token slot, or a match
// reaching behind a segment start returns 1: the caller then decodes the
// stream with one wave (inflate.hip), which also yields the reference's
// exact error.  Results are identical to the sequential decode by
// construction.  Replaces src/RawInflate.ts:127-143 for such streams.
#include <chrono>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>
#include <rocprim/warp/warp_scan.hpp>

#include "zt_internal.h"

namespace zt {

namespace {

constexpr uint32_t kMaxSync = 1u << 22;

// ZT_INF_DEBUG=1: report why a stream left the two-phase path
bool inf_debug() {
  static const bool on = getenv("ZT_INF_DEBUG") != nullptr;
  return on;
}
#define FALLBACK(...)                                   \
  do {                                                  \
    if (inf_debug()) fprintf(stderr, "[zt inflate] " __VA_ARGS__); \
    return 1;                                           \
  } while (0)
#ifndef ZT_DF_BLOCK
#define ZT_DF_BLOCK 32768
#endif
#ifndef ZT_DF_GROUP
#define ZT_DF_GROUP 1
#endif
// this engine's units are one DEFLATE block of ZT_DF_GROUP parse blocks
// (deflate.hip): <= 1 token per byte
constexpr uint32_t kUnitTokCap = ZT_DF_BLOCK * ZT_DF_GROUP + 64;
static_assert(kUnitTokCap < (1u << 30), "token counts stay below TokResult::ntok's flag bits");

// sync point = byte after an aligned 00 00 FF FF; list entry = pos << 1 | restart
// One 16-byte aligned chunk per lane, loaded as one 16-byte word; the 8 bytes
// before it and the 12 after come from the neighbouring lanes (lanes at a
// wave's edge load them).  A sync point is 00 00 FF FF (u32 0xFFFF0000 at the
// candidate) ending at p; a restart point is the double marker
// 00 00 00 FF FF 00 | 00 00 FF FF before it.
__device__ __forceinline__ uint32_t fs_word(const uint8_t *in, uint64_t n, int64_t q) {
  // 4 bytes at q (bytes outside [0, n) read as 1: never part of a pattern)
  uint32_t v = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int64_t x = q + k;
    v |= (uint32_t)((x >= 0 && (uint64_t)x < n) ? in[x] : 1) << (8 * k);
  }
  return v;
}
#ifndef ZT_FS_ITER
#define ZT_FS_ITER 8  // 4 / 8 / 16: 0.305 / 0.256 / 0.337 ms per GiB (each workgroup's one atomic on the shared counter; gpurun_out/r05ay)
#endif
constexpr uint32_t FS_ITER = ZT_FS_ITER;  // 4 KiB spans per workgroup (fewer, longer workgroups)
constexpr uint32_t kFsLocal = 64;  // sync candidates a workgroup gathers before its one global atomic
// Workgroup k appends to list region k % FS_SPLIT (its own counter, in its own
// 128-byte line): one counter took every workgroup's atomic, serialised where
// device-scope atomics execute; fs_gather then packs the regions
#ifndef ZT_FS_SPLIT
#define ZT_FS_SPLIT 64
#endif
constexpr uint32_t FS_SPLIT = ZT_FS_SPLIT;
constexpr uint32_t kFsRegion = kMaxSync / FS_SPLIT;  // candidates per region (more: the stream leaves this path)
constexpr uint32_t kFsCountStride = 32;             // u32 counters 128 bytes apart
#ifndef ZT_FS_NT
#define ZT_FS_NT 1
#endif
__global__ __launch_bounds__(256) void find_syncs(const uint8_t *__restrict__ in, uint64_t lo, uint64_t n,
                                                  uint64_t *__restrict__ list, uint32_t *__restrict__ count) {
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  const int lane = threadIdx.x & 63;
  uint32_t *rcount = count + (blockIdx.x % FS_SPLIT) * kFsCountStride;
  uint64_t *rlist = list + (uint64_t)(blockIdx.x % FS_SPLIT) * kFsRegion;
  __shared__ uint32_t s_n, s_base;
  __shared__ uint64_t s_list[kFsLocal];
  if (threadIdx.x == 0) s_n = 0;
  __syncthreads();
  // A wave scans FS_ITER contiguous KiB (1 KiB per step, 16 bytes per lane):
  // the bytes around a lane's chunk come from its neighbours, across steps
  // from the previous step's lane 63 / the next step's lane 0, and only the
  // wave's two ends are loaded apart -- with the chunks, all in flight at once
  const uint32_t wv = threadIdx.x >> 6;
  const uint64_t wbase = (lo & ~uint64_t(15)) + ((uint64_t)blockIdx.x * FS_ITER * 256 + (uint64_t)wv * FS_ITER * 64) * 16;
  const bool in16 = (reinterpret_cast<uintptr_t>(in) & 15) == 0;
  const bool aligned = (reinterpret_cast<uintptr_t>(in) & 3) == 0;
  const uint32_t *in32 = reinterpret_cast<const uint32_t *>(in);
  auto edge = [&](int64_t q) -> uint32_t {  // 4 bytes at q, as fs_word
    return aligned && q >= 0 && (uint64_t)q + 4 <= n ? in32[q / 4] : fs_word(in, n, q);
  };
  u32x4 pre[FS_ITER];
#pragma unroll
  for (uint32_t it = 0; it < FS_ITER; ++it) {
    const uint64_t base = wbase + ((uint64_t)it * 64 + lane) * 16;
    pre[it] = base + 16 <= n && in16
                  ? (ZT_FS_NT ? __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(in + base))
                             : *reinterpret_cast<const u32x4 *>(in + base))
                  : u32x4{0u, 0u, 0u, 0u};
  }
  // lane 0: the 8 bytes before the wave's span; lane 63: the 12 after it
  uint32_t e0 = 0, e1 = 0, e2 = 0;
  if (lane == 0) {
    e0 = edge((int64_t)wbase - 8);
    e1 = edge((int64_t)wbase - 4);
  }
  if (lane == 63) {
    const int64_t q = (int64_t)(wbase + (uint64_t)FS_ITER * 1024);
    e0 = edge(q);
    e1 = edge(q + 4);
    e2 = edge(q + 8);
  }
  uint32_t c0 = e0, c1 = e1;  // lane 0: the 8 bytes before this step's chunk
#pragma unroll
  for (uint32_t it = 0; it < FS_ITER; ++it) {
  const uint64_t base = wbase + ((uint64_t)it * 64 + lane) * 16;
  // words: w[0..1] = bytes [base - 8, base), w[2..5] = [base, base + 16), w[6..8] = [base + 16, base + 28)
  uint32_t w[9];
  const bool whole = base + 16 <= n && in16;
  if (whole) {
    const u32x4 v = pre[it];
    w[2] = v.x;
    w[3] = v.y;
    w[4] = v.z;
    w[5] = v.w;
  } else {
#pragma unroll
    for (int k = 0; k < 4; ++k) w[2 + k] = fs_word(in, n, (int64_t)base + 4 * k);
  }
  w[0] = (uint32_t)__shfl_up((int)w[4], 1, 64);
  w[1] = (uint32_t)__shfl_up((int)w[5], 1, 64);
  w[6] = (uint32_t)__shfl_down((int)w[2], 1, 64);
  w[7] = (uint32_t)__shfl_down((int)w[3], 1, 64);
  w[8] = (uint32_t)__shfl_down((int)w[4], 1, 64);
  if (lane == 0) {
    w[0] = c0;
    w[1] = c1;
  }
  c0 = (uint32_t)__builtin_amdgcn_readlane((int)w[4], 63);
  c1 = (uint32_t)__builtin_amdgcn_readlane((int)w[5], 63);
  if (it + 1 < FS_ITER) {
    // the next step's first 12 bytes: lane 0's chunk there when it is whole
    const uint64_t nb = wbase + (uint64_t)(it + 1) * 1024;
    const bool nwhole = nb + 16 <= n && in16;
    const uint32_t x0 = (uint32_t)__builtin_amdgcn_readlane((int)pre[it + 1].x, 0);
    const uint32_t x1 = (uint32_t)__builtin_amdgcn_readlane((int)pre[it + 1].y, 0);
    const uint32_t x2 = (uint32_t)__builtin_amdgcn_readlane((int)pre[it + 1].z, 0);
    if (lane == 63) {
      w[6] = nwhole ? x0 : fs_word(in, n, (int64_t)nb);
      w[7] = nwhole ? x1 : fs_word(in, n, (int64_t)nb + 4);
      w[8] = nwhole ? x2 : fs_word(in, n, (int64_t)nb + 8);
    }
  } else if (lane == 63) {
    w[6] = e0;
    w[7] = e1;
    w[8] = e2;
  }
  if (base >= n) continue;
  auto at = [&](int x) -> uint32_t {  // 4 bytes at base - 8 + x (0 <= x <= 32)
    return (x & 3) ? __builtin_amdgcn_alignbyte(w[(x >> 2) + 1], w[x >> 2], x & 3) : w[x >> 2];
  };
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    if (at(8 + j) == 0xFFFF0000u) {
      const uint64_t p = base + j + 4;
      if (p > lo && p < n) {
        // bytes base + j - 6 .. base + j - 1: 00 00 00 FF FF 00
        const bool restart = base + j >= 6 && at(2 + j) == 0xFF000000u && (at(6 + j) & 0xFFFFu) == 0x00FFu;
        // gathered per workgroup (one global atomic per workgroup)
        const uint64_t v = (p << 1) | (restart ? 1 : 0);
        const uint32_t k = atomicAdd(&s_n, 1u);
        if (k < kFsLocal) {
          s_list[k] = v;
        } else {
          const uint32_t g = atomicAdd(rcount, 1u);
          if (g < kFsRegion) rlist[g] = v;
        }
      }
    }
  }
  }
  __syncthreads();
  const uint32_t m = s_n < kFsLocal ? s_n : kFsLocal;
  if (threadIdx.x == 0 && m) s_base = atomicAdd(rcount, m);
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < m; i += 256)
    if (s_base + i < kFsRegion) rlist[s_base + i] = s_list[i];
}

// the FS_SPLIT regions of find_syncs packed into `out` (region order; the
// sort that follows makes the order irrelevant), one workgroup per region;
// *total = the candidates, or kMaxSync + 1 when a region overflowed
__global__ __launch_bounds__(256) void fs_gather(const uint64_t *__restrict__ list, const uint32_t *__restrict__ count,
                                                 uint64_t *__restrict__ out, uint32_t *__restrict__ total) {
  const uint32_t r = blockIdx.x;
  __shared__ uint32_t s_off, s_over;
  if (threadIdx.x < 64) {
    uint32_t below = 0, all = 0, over = 0;
    for (uint32_t q = threadIdx.x; q < FS_SPLIT; q += 64) {
      const uint32_t c = count[q * kFsCountStride];
      over |= c > kFsRegion ? 1u : 0u;
      all += c;
      below += q < r ? c : 0u;
    }
    for (int o = 32; o; o >>= 1) {
      below += (uint32_t)__shfl_xor((int)below, o, 64);
      all += (uint32_t)__shfl_xor((int)all, o, 64);
      over |= (uint32_t)__shfl_xor((int)over, o, 64);
    }
    if (threadIdx.x == 0) {
      s_off = below;
      s_over = over;
      if (r == 0) *total = over ? kMaxSync + 1 : all;
    }
  }
  __syncthreads();
  if (s_over) return;
  const uint32_t c = count[r * kFsCountStride];
  const uint64_t *src = list + (uint64_t)r * kFsRegion;
  for (uint32_t i = threadIdx.x; i < c; i += 256) out[s_off + i] = src[i];
}

size_t align256(size_t v) { return (v + 255) & ~size_t(255); }

// sorted candidates (pos << 1 | restart) -> first of each position
__global__ __launch_bounds__(256) void unit_flags(const uint64_t *__restrict__ key, uint32_t cnt,
                                                  uint32_t *__restrict__ flag) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i > cnt) return;
  flag[i] = i < cnt && (i == 0 || (key[i] >> 1) != (key[i - 1] >> 1)) ? 1u : 0u;
}

// unit k + 1 starts at the k-th distinct sync point (unit 0 at `index`);
// pos[cnt] = the number of distinct sync points.  Token slot of a unit: every
// token takes at least one input bit, and a real unit ends at the next real
// sync point, so min(cap, 8 x the bytes up to the next candidate + 64)
// holds it (a false candidate inside a real unit's block can only make that
// unit overflow its slot: the stream then leaves this path).  Without the
// bound, every one of a crafted input's dense false candidates took a whole
// block's slot (~128 KiB each).
__global__ __launch_bounds__(256) void unit_jobs(const uint64_t *__restrict__ key, const uint32_t *__restrict__ flag,
                                                 const uint32_t *__restrict__ pos, uint32_t cnt, uint64_t n,
                                                 uint64_t index, uint32_t cap, uint64_t *__restrict__ sync,
                                                 uint8_t *__restrict__ restart, TokJob *__restrict__ jobs,
                                                 uint64_t *__restrict__ slot, uint32_t *__restrict__ nrestart,
                                                 uint32_t *__restrict__ span_key, uint32_t *__restrict__ unit_id) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  auto job = [&](uint32_t u, uint64_t start, uint64_t next) {
    // (launch order: the longest input span first -- sorted on a 20-bit
    // key, spans of 1 MiB and more tied first)
    const uint64_t span = next > start ? next - start : 0;
    if (span_key) {
      span_key[u] = 0xFFFFFu - (uint32_t)(span < 0xFFFFFull ? span : 0xFFFFFull);
      unit_id[u] = u;
    }
    TokJob j;
    j.start = start;
    j.tok_off = 0;  // unit_slots
    const uint64_t room = (next > start ? next - start : 0) * 8 + 64;
    j.tok_cap = (uint32_t)(room < cap ? room : cap);
    j.stop_first = u;  // sync[u] is the first sync point after start
    j.end = 0;
    jobs[u] = j;
    slot[u] = (j.tok_cap + 63) & ~63u;
  };
  if (i == 0) job(0, index, cnt ? key[0] >> 1 : n);
  if (i >= cnt || !flag[i]) return;
  const uint32_t k = pos[i];
  const uint64_t p = key[i] >> 1;
  uint32_t j = i + 1;
  while (j < cnt && (key[j] >> 1) == p) ++j;
  sync[k] = p;
  restart[k] = (uint8_t)(key[i] & 1);
  if (key[i] & 1) atomicAdd(nrestart, 1u);
  job(k + 1, p, j < cnt ? key[j] >> 1 : n);
}

// token offsets = exclusive scan of the slots; total[0] = all slots
__global__ __launch_bounds__(256) void unit_slots(const uint64_t *__restrict__ off, const uint64_t *__restrict__ slot,
                                                  const uint32_t *__restrict__ nunits_m1, TokJob *__restrict__ jobs,
                                                  uint64_t *__restrict__ total) {
  const uint32_t u = blockIdx.x * 256 + threadIdx.x;
  const uint32_t units = *nunits_m1 + 1;
  if (u >= units) return;
  jobs[u].tok_off = off[u];
  if (u + 1 == units) total[0] = off[u] + slot[u];
}

}  // namespace

// ---- the chain on the device (the common case) --------------------------------
// When every unit is on the chain in order -- unit u stops at sync point u and
// the last one at BFINAL, i.e. no false sync-point candidate -- the chain, its
// copy segments and their descriptor offsets are prefix sums, and one
// workgroup builds them where the host walk needed every unit's result back
// over PCIe and the chain sent down again (a host round trip between tokenize
// and expand).  Anything else (a false candidate, a unit error, an output past
// the capacity, more segments than the bound) leaves info->ok = 0: expand and
// copy return at once and the host walks the chain as before.  Segment rules
// as the host walk's: a segment starts at unit 0 and at the first unit after
// a restart point that has output bytes since the previous restart point
// (empty segments merge into the next); its descriptors start 512-aligned; a
// segment of stored runs only is copied by expand_kernel (SegJob count bit 31).
constexpr int CH_T = 1024;
constexpr uint32_t CH_MAXU = 40960;  // units (LDS: 2 B each): 1.25 GiB of 32 KiB blocks
constexpr int CH_B = 8;              // rounds whose loads are in flight together
constexpr uint32_t CH_MAXS = 2048;   // segments (LDS)

__device__ __forceinline__ uint64_t shfl_up64(uint64_t v, int d) {
  const uint32_t lo = (uint32_t)__shfl_up((int)(uint32_t)v, d, 64);
  const uint32_t hi = (uint32_t)__shfl_up((int)(uint32_t)(v >> 32), d, 64);
  return ((uint64_t)hi << 32) | lo;
}
struct AddU64 {
  __device__ uint64_t operator()(uint64_t a, uint64_t b) const { return a + b; }
};
struct MaxU64 {
  __device__ uint64_t operator()(uint64_t a, uint64_t b) const { return a > b ? a : b; }
};
// exclusive scan over the workgroup's CH_T threads (identity 0); *total = the reduction
template <typename Op>
__device__ uint64_t block_excl_scan(uint64_t v, Op op, uint64_t *wsum, uint64_t *total) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint64_t x = v;
  for (int d = 1; d < 64; d <<= 1) {
    const uint64_t y = shfl_up64(x, d);
    if (lane >= d) x = op(x, y);
  }
  if (lane == 63) wsum[w] = x;
  __syncthreads();
  if (w == 0) {
    uint64_t sw = lane < CH_T / 64 ? wsum[lane] : 0;
    for (int d = 1; d < CH_T / 64; d <<= 1) {
      const uint64_t y = shfl_up64(sw, d);
      if (lane >= d) sw = op(sw, y);
    }
    if (lane < CH_T / 64) wsum[lane] = sw;
  }
  __syncthreads();
  uint64_t ex = shfl_up64(x, 1);
  if (lane == 0) ex = 0;
  const uint64_t r = op(w ? wsum[w - 1] : 0, ex);
  if (total) *total = wsum[CH_T / 64 - 1];
  __syncthreads();
  return r;
}

// wave w owns units [w * wu, (w + 1) * wu), taken 64 at a time (lane = unit:
// every global access coalesced); running values cross rounds in registers
// and waves through one workgroup scan
__global__ __launch_bounds__(CH_T) void chain_kernel(const TokResult *__restrict__ res, const uint8_t *__restrict__ restart,
                                                     const uint64_t *__restrict__ tok_off, uint32_t units,
                                                     uint64_t out_cap, uint64_t desc_cap, uint32_t max_seg,
                                                     ChainUnit *__restrict__ cu, SegJob *__restrict__ sj,
                                                     ChainInfo *__restrict__ info, uint32_t *__restrict__ ekey,
                                                     uint32_t *__restrict__ eid) {
  __shared__ uint16_t ol[CH_MAXU];              // unit output bytes (<= 65535 here)
  __shared__ uint32_t candb[CH_MAXU / 32];      // unit follows a restart point (or is unit 0)
  __shared__ uint32_t dirb[CH_MAXU / 32];       // unit is stored runs only, or empty
  __shared__ uint64_t seg_off[CH_MAXS + 1];     // output offset of segment k's first unit; [nseg] = total
  __shared__ uint64_t seg_desc[CH_MAXS];
  __shared__ uint32_t seg_first[CH_MAXS + 1];
  __shared__ uint32_t seg_direct[CH_MAXS];
  __shared__ uint64_t wsum[CH_T / 64];
  __shared__ int bad;
  const uint32_t t = threadIdx.x;
  const int lane = t & 63;
  const uint32_t w = t >> 6, nw = CH_T / 64;
  const uint32_t wu = ((units + nw - 1) / nw + 63) & ~63u;  // units per wave, whole rounds
  const uint32_t w0 = w * wu < units ? w * wu : units, w1 = w0 + wu < units ? w0 + wu : units;
  if (t == 0) bad = 0;
  for (uint32_t i = t; i < CH_MAXU / 32; i += CH_T) candb[i] = dirb[i] = 0;
  for (uint32_t i = t; i < CH_MAXS; i += CH_T) seg_direct[i] = 1;
  __syncthreads();
  // A: the unit results into LDS (CH_B rounds' loads in flight); every unit
  // on the chain in order; the wave's bytes
  bool ok = true;
  uint64_t wlen = 0;
  for (uint32_t r0 = w0; r0 < w1; r0 += 64 * CH_B) {
    uint64_t olen[CH_B];
    int32_t st[CH_B], stop[CH_B];
    uint32_t ntok[CH_B];
    uint8_t rs[CH_B];
#pragma unroll
    for (int j = 0; j < CH_B; ++j) {
      const uint32_t v = r0 + 64 * j + lane, u = v < w1 ? v : w0;
      olen[j] = res[u].out_len;
      st[j] = res[u].status;
      stop[j] = res[u].stop_idx;
      ntok[j] = res[u].ntok;
      rs[j] = restart[u ? u - 1 : 0];
    }
#pragma unroll
    for (int j = 0; j < CH_B; ++j) {
      const uint32_t u = r0 + 64 * j + lane;
      if (u >= w1) continue;
      ok = ok && st[j] == ZT_OK && olen[j] <= 0xFFFFull && (u + 1 < units ? stop[j] == (int32_t)u : stop[j] < 0);
      ol[u] = (uint16_t)olen[j];
      wlen += olen[j];
      if (u == 0 || rs[j] != 0) atomicOr(&candb[u >> 5], 1u << (u & 31));
      if ((ntok[j] >> 30) == 3u || olen[j] == 0) atomicOr(&dirb[u >> 5], 1u << (u & 31));
    }
  }
  if (!ok) bad = 1;
  for (int o = 32; o; o >>= 1) wlen += ((uint64_t)(uint32_t)__shfl_xor((int)(uint32_t)(wlen >> 32), o, 64) << 32) |
                                       (uint32_t)__shfl_xor((int)(uint32_t)wlen, o, 64);
  uint64_t total;
  const uint64_t wbase = block_excl_scan(lane == 0 ? wlen : 0, AddU64(), wsum, &total);  // (one lane per wave)
  const uint64_t base = __shfl((int)(uint32_t)wbase, 0, 64) | ((uint64_t)(uint32_t)__shfl((int)(uint32_t)(wbase >> 32), 0, 64) << 32);
  auto cand = [&](uint32_t u) { return u < w1 && ((candb[u >> 5] >> (u & 31)) & 1u); };
  // One round of 64 units: u's output offset o (the round's sums are 32-bit:
  // units <= 65535 bytes), whether u starts a segment (a restart point with
  // output since the previous one: pcr = that one's offset before the round),
  // and the running values for the next round (wave scans by DPP, rocPRIM).
  using WScan = rocprim::warp_scan<uint32_t, 64>;
  __shared__ typename WScan::storage_type wst[CH_T / 64];
  struct Round {
    uint64_t o;
    bool start;
  };
  auto round = [&](uint32_t u, uint32_t l, uint64_t &off, uint64_t &pcr) -> Round {
    uint32_t inc;
    WScan().inclusive_scan(l, inc, wst[w], rocprim::plus<uint32_t>());
    const uint64_t o = off + inc - l;
    const bool c = cand(u);
    const uint32_t cv = c ? inc - l + 1 : 0u;  // 1 + the round-local offset of a restart point
    uint32_t ex;
    WScan().exclusive_scan(cv, ex, 0u, wst[w], rocprim::maximum<uint32_t>());
    const uint64_t before = ex ? off + ex - 1 : pcr;
    const uint32_t rmax = (uint32_t)__shfl((int)(ex > cv ? ex : cv), 63, 64);
    const bool start = u < w1 && (u == 0 || (c && o > before));
    if (rmax) pcr = off + rmax - 1;
    off += (uint32_t)__shfl((int)inc, 63, 64);
    return Round{o, start};
  };
  // B: output offset of the wave's last restart point (non-decreasing: a max-scan)
  uint64_t off = base, last = 0;
  for (uint32_t r0 = w0; r0 < w1; r0 += 64) {
    const uint32_t u = r0 + lane;
    (void)round(u, u < w1 ? ol[u] : 0u, off, last);
  }
  const uint64_t prevw = block_excl_scan(lane == 0 ? last : 0, MaxU64(), wsum, nullptr);
  const uint64_t prev = __shfl((int)(uint32_t)prevw, 0, 64) | ((uint64_t)(uint32_t)__shfl((int)(uint32_t)(prevw >> 32), 0, 64) << 32);
  // C: segment starts per wave
  uint64_t nstart = 0, pc = prev;
  off = base;
  for (uint32_t r0 = w0; r0 < w1; r0 += 64) {
    const uint32_t u = r0 + lane;
    const Round r = round(u, u < w1 ? ol[u] : 0u, off, pc);
    nstart += __popcll(__ballot(r.start));
  }
  uint64_t nseg64;
  const uint64_t sbw = block_excl_scan(lane == 0 ? nstart : 0, AddU64(), wsum, &nseg64);
  const uint32_t sbase = (uint32_t)__shfl((int)(uint32_t)sbw, 0, 64);
  const uint32_t nseg = (uint32_t)nseg64;
  if (bad || total > out_cap || nseg > max_seg || nseg > CH_MAXS) {
    if (t == 0) info->ok = 0;
    return;  // (uniform: bad was set before the scans' barriers)
  }
  // D: the segment table; a segment is direct when all its units are stored runs (or empty)
  uint32_t k = sbase;  // segments started before this round
  pc = prev;
  off = base;
  for (uint32_t r0 = w0; r0 < w1; r0 += 64) {
    const uint32_t u = r0 + lane;
    const Round r = round(u, u < w1 ? ol[u] : 0u, off, pc);
    const uint64_t sm = __ballot(r.start);
    const uint32_t g = k + (uint32_t)__popcll(sm & ((2ull << lane) - 1)) - 1;  // this unit's segment
    if (r.start) {
      seg_first[g] = u;
      seg_off[g] = r.o;
    }
    if (u < w1 && !((dirb[u >> 5] >> (u & 31)) & 1)) seg_direct[g] = 0;
    k += (uint32_t)__popcll(sm);
  }
  if (t == 0) {
    seg_first[nseg] = units;
    seg_off[nseg] = total;
  }
  __syncthreads();
  // E: descriptor offsets, each segment 512-aligned
  const uint32_t sper = (nseg + CH_T - 1) / CH_T;
  const uint32_t s0 = t * sper < nseg ? t * sper : nseg, s1 = s0 + sper < nseg ? s0 + sper : nseg;
  uint64_t dl = 0;
  for (uint32_t q = s0; q < s1; ++q) dl += (seg_off[q + 1] - seg_off[q] + 511) & ~uint64_t(511);
  uint64_t db = block_excl_scan(dl, AddU64(), wsum, nullptr);
  for (uint32_t q = s0; q < s1; ++q) {
    seg_desc[q] = db;
    db += (seg_off[q + 1] - seg_off[q] + 511) & ~uint64_t(511);
  }
  __syncthreads();
  const uint64_t desc_total = seg_desc[nseg - 1] + (total - seg_off[nseg - 1]);
  if (desc_total + 1024 > desc_cap) {
    if (t == 0) info->ok = 0;
    return;  // (uniform)
  }
  // F: chain units (coalesced) and segment jobs
  k = sbase;
  pc = prev;
  off = base;
  for (uint32_t b0 = w0; b0 < w1; b0 += 64 * CH_B) {
    uint64_t to[CH_B];
    uint32_t nt[CH_B];
#pragma unroll
    for (int j = 0; j < CH_B; ++j) {  // CH_B rounds' loads in flight (each round waited alone: 0.1 ms)
      const uint32_t v = b0 + 64 * j + lane, uu = v < w1 ? v : w0;
      to[j] = tok_off[uu];
      nt[j] = res[uu].ntok;
    }
#pragma unroll
    for (int j = 0; j < CH_B; ++j) {
      const uint32_t r0 = b0 + 64 * j;
      if (r0 >= w1) break;  // (wave-uniform)
      const uint32_t u = r0 + lane;
      const uint32_t l = u < w1 ? ol[u] : 0u;
      const Round r = round(u, l, off, pc);
      const uint64_t sm = __ballot(r.start);
      const uint32_t g = k + (uint32_t)__popcll(sm & ((2ull << lane) - 1)) - 1;
      if (u < w1) {
        ChainUnit x;
        x.tok_off = to[j];
        x.out_off = r.o;
        x.seg_off = seg_off[g];
        x.desc_off = seg_desc[g] + (r.o - seg_off[g]);
        x.ntok = seg_direct[g] ? nt[j] : (nt[j] & ~0x40000000u);
        x.out_len = l;
        cu[u] = x;
        if (ekey) {  // expand's launch order: most tokens first (17-bit key)
          const uint32_t nt = x.ntok & 0x3FFFFFFFu;
          ekey[u] = 0x1FFFFu - (nt < 0x1FFFFu ? nt : 0x1FFFFu);
          eid[u] = u;
        }
      }
      k += (uint32_t)__popcll(sm);
    }
  }
  for (uint32_t q = t; q < nseg; q += CH_T)
    sj[q] = SegJob{seg_first[q], (seg_first[q + 1] - seg_first[q]) | (seg_direct[q] ? 0x80000000u : 0u)};
  if (t == 0) {
    info->ok = 1;
    info->nseg = nseg;
    info->total = total;
    info->end_bits = res[units - 1].end_bits;
    info->desc_total = desc_total;
  }
}

// ZT_INF_TIMING=1: host wall time of inflate_segments_dev's stages on stderr (measurement only)
static double it_now() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
#define IT(label)                                                   \
  do {                                                              \
    static const bool on_ = getenv("ZT_INF_TIMING") != nullptr;     \
    if (on_) fprintf(stderr, "[inflate] %-24s %9.3f ms\n", label, it_now()); \
  } while (0)

// a unit of the chain starts at byte `pos` (the device chain: every unit is
// on it); flag[0] |= 1 then
__global__ void unit_starts_at(const TokJob *__restrict__ jobs, uint32_t units, uint64_t pos, uint32_t *flag) {
  for (uint32_t u = blockIdx.x * blockDim.x + threadIdx.x; u < units; u += gridDim.x * blockDim.x)
    if (jobs[u].start == pos) atomicOr(flag, 1u);
}

int inflate_segments_dev(DeviceCtx *c, const uint8_t *d_in, size_t n, size_t index, uint8_t **d_out_io,
                         size_t out_cap, size_t *out_len, size_t *end_ip, hipStream_t s, uint64_t boundary) {
  IT("start");
  if (n < index + (1u << 14)) return 1;  // small: one wave is as fast
  // 1. sync points
  void *d_cand;
  // [counters: FS_SPLIT lines | total][regions: kMaxSync][packed: kMaxSync]
  constexpr size_t kCntBytes = (size_t)FS_SPLIT * kFsCountStride * 4 + 256;
  ZT_TRY(scratch(c, 5, kCntBytes + 2 * (size_t)kMaxSync * 8, &d_cand));
  uint32_t *d_rcount = static_cast<uint32_t *>(d_cand);
  uint32_t *d_count = d_rcount + (size_t)FS_SPLIT * kFsCountStride;
  uint64_t *d_regions = reinterpret_cast<uint64_t *>(static_cast<uint8_t *>(d_cand) + kCntBytes);
  uint64_t *d_list = d_regions + kMaxSync;
  ZT_HIP(hipMemsetAsync(d_rcount, 0, (size_t)FS_SPLIT * kFsCountStride * 4, s));
  const uint64_t span = n - (index & ~size_t(15));
  const uint32_t grid = (uint32_t)((span + 16 * 256 * FS_ITER - 1) / (16 * 256 * FS_ITER));
  ZT_TRY(timing_begin(c, s, 2));
  find_syncs<<<grid, 256, 0, s>>>(d_in, index, n, d_regions, d_rcount);
  ZT_HIP(hipGetLastError());
  fs_gather<<<FS_SPLIT, 256, 0, s>>>(d_regions, d_rcount, d_list, d_count);
  ZT_HIP(hipGetLastError());
  uint32_t cnt = 0;
  ZT_TRY(readback(c, &cnt, d_count, 4, s));
  IT("sync points counted");
  if (cnt == 0 || cnt > kMaxSync) FALLBACK("%u sync points\n", cnt);
  // 2. the candidates sorted, deduplicated and turned into units on the
  // device (rocPRIM radix sort + scan): unit 0 starts at `index`, unit k + 1
  // at the k-th sync point
  int end_bit = 1;
  while (end_bit < 64 && ((uint64_t)n << 1 | 1) >> end_bit) ++end_bit;
  const size_t units_max = (size_t)cnt + 1;
  size_t t_sort = 0, t_scan = 0, t_scan64 = 0;
  ZT_HIP(rocprim::radix_sort_keys(nullptr, t_sort, (const uint64_t *)nullptr, (uint64_t *)nullptr, (size_t)cnt, 0u,
                                  (unsigned)end_bit, s));
  ZT_HIP(rocprim::exclusive_scan(nullptr, t_scan, (const uint32_t *)nullptr, (uint32_t *)nullptr, 0u, units_max,
                                 rocprim::plus<uint32_t>(), s));
  ZT_HIP(rocprim::exclusive_scan(nullptr, t_scan64, (const uint64_t *)nullptr, (uint64_t *)nullptr, (uint64_t)0,
                                 units_max, rocprim::plus<uint64_t>(), s));
  const size_t t_bytes = align256(std::max(t_sort, std::max(t_scan, t_scan64)));
  const size_t key_bytes = align256((size_t)cnt * 8), flag_bytes = align256(units_max * 4);
  const size_t slot_bytes = align256(units_max * 8);
  void *d_sort;
  ZT_TRY(scratch(c, 20, t_bytes + key_bytes + 2 * flag_bytes + 2 * slot_bytes + 256, &d_sort));
  uint8_t *sb = static_cast<uint8_t *>(d_sort);
  uint64_t *d_key = reinterpret_cast<uint64_t *>(sb + t_bytes);
  uint32_t *d_flag = reinterpret_cast<uint32_t *>(sb + t_bytes + key_bytes);
  uint32_t *d_pos = reinterpret_cast<uint32_t *>(sb + t_bytes + key_bytes + flag_bytes);
  uint64_t *d_slot = reinterpret_cast<uint64_t *>(sb + t_bytes + key_bytes + 2 * flag_bytes);
  uint64_t *d_off = d_slot + slot_bytes / 8;
  uint64_t *d_ttot = d_off + slot_bytes / 8;  // [0] token slots in all, [1] distinct sync points
  ZT_HIP(rocprim::radix_sort_keys(sb, t_sort, d_list, d_key, (size_t)cnt, 0u, (unsigned)end_bit, s));
  const uint32_t g = (cnt + 1 + 255) / 256;
  unit_flags<<<g, 256, 0, s>>>(d_key, cnt, d_flag);
  ZT_HIP(hipGetLastError());
  ZT_HIP(rocprim::exclusive_scan(sb, t_scan, d_flag, d_pos, 0u, units_max, rocprim::plus<uint32_t>(), s));
  const size_t stops_bytes = align256((size_t)cnt * 8);
  const size_t restart_bytes = align256(units_max);
  const size_t jobs_bytes = align256(units_max * sizeof(TokJob));
  const size_t res_bytes = align256(units_max * sizeof(TokResult));
  void *d_meta;
  ZT_TRY(scratch(c, 6, stops_bytes + restart_bytes + jobs_bytes + res_bytes, &d_meta));
  uint64_t *d_stops = static_cast<uint64_t *>(d_meta);
  uint8_t *d_restart = static_cast<uint8_t *>(d_meta) + stops_bytes;
  TokJob *d_jobs = reinterpret_cast<TokJob *>(static_cast<uint8_t *>(d_meta) + stops_bytes + restart_bytes);
  TokResult *d_res =
      reinterpret_cast<TokResult *>(static_cast<uint8_t *>(d_meta) + stops_bytes + restart_bytes + jobs_bytes);
  ZT_HIP(hipMemsetAsync(d_slot, 0, units_max * 8, s));
  ZT_HIP(hipMemsetAsync(d_ttot + 2, 0, 8, s));
  // tokenize launch order (slot 28): [span keys | unit ids | sorted keys |
  // sorted ids | sort storage]
  // (up to 128 K candidates: 4 GiB of 32 KiB blocks; a crafted stream of
  // dense false candidates keeps the position order and no order buffers)
  static const bool lpt_env = getenv("ZT_TOK_ORDER") ? atoi(getenv("ZT_TOK_ORDER")) != 0 : true;
  const bool lpt = lpt_env && units_max <= (1u << 17);
  size_t t_ord = 0;
  if (lpt)
    ZT_HIP(rocprim::radix_sort_pairs(nullptr, t_ord, (const uint32_t *)nullptr, (uint32_t *)nullptr,
                                     (const uint32_t *)nullptr, (uint32_t *)nullptr, units_max, 0u, 20u, s));
  const size_t ord_b = align256((lpt ? units_max : 1) * 4);
  void *d_ordbuf;
  ZT_TRY(scratch(c, 28, 4 * ord_b + align256(t_ord), &d_ordbuf));
  uint32_t *d_skey = static_cast<uint32_t *>(d_ordbuf);
  uint32_t *d_uid = reinterpret_cast<uint32_t *>(static_cast<uint8_t *>(d_ordbuf) + ord_b);
  uint32_t *d_skey2 = reinterpret_cast<uint32_t *>(static_cast<uint8_t *>(d_ordbuf) + 2 * ord_b);
  uint32_t *d_order = reinterpret_cast<uint32_t *>(static_cast<uint8_t *>(d_ordbuf) + 3 * ord_b);
  void *d_ordtmp = static_cast<uint8_t *>(d_ordbuf) + 4 * ord_b;
  unit_jobs<<<g, 256, 0, s>>>(d_key, d_flag, d_pos, cnt, n, index, kUnitTokCap, d_stops, d_restart, d_jobs, d_slot,
                              reinterpret_cast<uint32_t *>(d_ttot + 2), lpt ? d_skey : nullptr, d_uid);
  ZT_HIP(hipGetLastError());
  ZT_HIP(rocprim::exclusive_scan(sb, t_scan64, d_slot, d_off, (uint64_t)0, units_max, rocprim::plus<uint64_t>(), s));
  unit_slots<<<g, 256, 0, s>>>(d_off, d_slot, d_pos + cnt, d_jobs, d_ttot);
  ZT_HIP(hipGetLastError());
  uint64_t tot_h[3] = {0, 0, 0};
  {
    void *mb;
    ZT_TRY(mailbox(c, 24, &mb));
    uint64_t *m64 = static_cast<uint64_t *>(mb);
    m64[1] = m64[2] = 0;
    ZT_TRY(x_copy(&m64[0], d_ttot, 8, s));
    ZT_TRY(x_copy(&m64[1], d_pos + cnt, 4, s));
    ZT_TRY(x_copy(&m64[2], d_ttot + 2, 4, s));
    ZT_HIP(hipStreamSynchronize(s));
    for (int k = 0; k < 3; ++k) tot_h[k] = m64[k];
  }
  IT("units counted");
  const uint32_t nsync = (uint32_t)tot_h[1];
  const size_t units = (size_t)nsync + 1;
  // Every candidate sync point gets a token slot before the chain shows which
  // are real block boundaries; the slots are bounded by the input bits up to
  // the next candidate (unit_jobs), so all of them together stay below 8
  // tokens per input byte + 64 per candidate.  Past the device's free memory,
  // or when the slots cannot be allocated, the stream takes the general path.
  const size_t tok_bytes = ((size_t)tot_h[0] + 256) * 4;  // + slack: chunked token reads
  // (only asked when the cached slots are too small: hipMemGetInfo is a
  // driver round trip on every call otherwise)
  if (tok_bytes > c->buf_size[4]) {
    size_t mem_free = 0, mem_total = 0;
    ZT_HIP(hipMemGetInfo(&mem_free, &mem_total));
    if (tok_bytes > c->buf_size[4] + mem_free / 2) FALLBACK("%zu sync candidates: token slots over budget\n", units);
  }
  void *d_tok;
  if (scratch(c, 4, tok_bytes, &d_tok) != ZT_OK) FALLBACK("token slots (%zu B) not allocated\n", tok_bytes);
  // metadata comes back through pinned staging (slot 1):
  // [restart flags | results | token offsets | chain | segments | statuses]
  void *hp;
  const size_t meta_a = restart_bytes + res_bytes + slot_bytes;
  const size_t meta_b = align256(units_max * sizeof(ChainUnit)) + align256(units_max * sizeof(SegJob)) +
                        2 * align256(units_max * 4);
  ZT_TRY(pinned(c, meta_a + meta_b, &hp, 1));
  uint8_t *pin = static_cast<uint8_t *>(hp);
  const uint8_t *restart = pin;
  // longest units first: the kernel's last units are short ones, so its tail
  // (SIMDs idle while the last units finish) is short
  if (lpt && units > 1)
    ZT_HIP(rocprim::radix_sort_pairs(d_ordtmp, t_ord, d_skey, d_skey2, d_uid, d_order, units, 0u, 20u, s));
  TokParams tp;
  tp.in = d_in;
  tp.n = n;
  tp.order = lpt && units > 1 ? d_order : nullptr;
  tp.stops = d_stops;
  tp.nstops = nsync;
  tp.jobs = d_jobs;
  tp.res = d_res;
  tp.tokens = static_cast<uint32_t *>(d_tok);
  tp.count = (uint32_t)units;
  static const char *simt_env = getenv("ZT_TOK_SIMT");
  tp.simt = simt_env ? atoi(simt_env) != 0 : 1;
  const bool check = getenv("ZT_TOK_CHECK") != nullptr;
  tp.dbg = nullptr;
  if (check) {
    void *d_dbg;
    ZT_TRY(scratch(c, 2, units * 64 + 8 * 64 * 32, &d_dbg));
    ZT_HIP(hipMemsetAsync(d_dbg, 0, units * 64 + 8 * 64 * 32, s));
    tp.dbg = static_cast<uint64_t *>(d_dbg);
  }
  tp.dump_unit = getenv("ZT_TOK_DUMP") ? (uint32_t)atoi(getenv("ZT_TOK_DUMP")) : 0xFFFFFFFFu;
  tp.dump_once = 0;
  tp.run_tokens = 1;
  ZT_TRY(timing_begin(c, s, 3));
  ZT_TRY(tokenize_units_dev(tp, s));
  ZT_TRY(timing_end(c, s, 3));
  // 3a. the common case: chain, segments and the resolve kernels straight on
  // the device (a caller-owned output: its capacity bounds the descriptors);
  // ZT_INF_HOST_CHAIN=1 forces the host walk (measurement)
  static const bool host_chain = getenv("ZT_INF_HOST_CHAIN") != nullptr;
  const uint32_t max_seg = (uint32_t)std::min<uint64_t>(tot_h[2] + 1, units);
  const uint64_t desc_cap = (uint64_t)out_cap + 512ull * max_seg + 2048;
  // The descriptors are sized from the caller's capacity here (the decoded
  // size is known only after the chain), and the scratch cache only grows: a
  // generous capacity takes the device chain only when its descriptors fit
  // what slot 3 already holds or 8 bytes per input byte (output up to 4x the
  // input); otherwise, and when the slot cannot grow, the host walks the chain
  // and sizes them from the real total.
  const bool desc_fits = desc_cap * 2 <= c->buf_size[3] || desc_cap * 2 <= 8ull * n + 4ull * (512ull * max_seg + 2048);
  if (*d_out_io && !check && !inf_debug() && !host_chain && max_seg <= CH_MAXS && units <= CH_MAXU &&
      out_cap <= (64ull << 30) && desc_fits) {
    void *d_chain, *d_desc;
    const size_t chain_bytes = align256(units * sizeof(ChainUnit)), seg_bytes = align256(max_seg * sizeof(SegJob));
    const size_t ust_bytes = align256(units * 4), st_bytes = align256(max_seg * 4);
    ZT_TRY(scratch(c, 7, chain_bytes + seg_bytes + ust_bytes + st_bytes + 512, &d_chain));
    if (scratch(c, 3, desc_cap * 2, &d_desc) != ZT_OK) {
      (void)hipGetLastError();  // (the failed allocation's sticky error)
      goto host_walk;
    }
    uint8_t *cb = static_cast<uint8_t *>(d_chain);
    ChainUnit *d_cu = reinterpret_cast<ChainUnit *>(cb);
    SegJob *d_sj = reinterpret_cast<SegJob *>(cb + chain_bytes);
    int32_t *d_ust = reinterpret_cast<int32_t *>(cb + chain_bytes + seg_bytes);
    int32_t *d_st = reinterpret_cast<int32_t *>(cb + chain_bytes + seg_bytes + ust_bytes);
    ChainInfo *d_info = reinterpret_cast<ChainInfo *>(cb + chain_bytes + seg_bytes + ust_bytes + st_bytes);
    uint32_t *d_bflag = reinterpret_cast<uint32_t *>(d_info + 1);
    if (boundary != ~0ull) {
      ZT_HIP(hipMemsetAsync(d_bflag, 0, 4, s));
      unit_starts_at<<<(uint32_t)std::min<size_t>(64, (units + 255) / 256), 256, 0, s>>>(d_jobs, (uint32_t)units,
                                                                                        boundary, d_bflag);
      ZT_HIP(hipGetLastError());
    }
    // (the tokenize order's buffers, free again, hold expand's: most tokens first)
    chain_kernel<<<1, CH_T, 0, s>>>(d_res, d_restart, d_off, (uint32_t)units, out_cap, desc_cap, max_seg, d_cu, d_sj,
                                    d_info, lpt ? d_skey : nullptr, d_uid);
    ZT_HIP(hipGetLastError());
    if (lpt && units > 1)
      ZT_HIP(rocprim::radix_sort_pairs(d_ordtmp, t_ord, d_skey, d_skey2, d_uid, d_order, units, 0u, 20u, s));
    ResolveParams rp;
    rp.tokens = static_cast<const uint32_t *>(d_tok);
    rp.units = d_cu;
    rp.segs = d_sj;
    rp.out = *d_out_io;
    rp.desc = static_cast<uint16_t *>(d_desc);
    rp.unit_status = d_ust;
    rp.seg_status = d_st;
    rp.nunits = (uint32_t)units;
    rp.nseg = max_seg;  // (grid; copy waves past info->nseg return at once)
    rp.marker = 0;
    rp.in = d_in;
    rp.info = d_info;
    rp.order = lpt && units > 1 ? d_order : nullptr;
    IT("device chain launched");
    ZT_TRY(resolve_segments_dev(rp, s));
    ZT_TRY(timing_end(c, s, 2));
    // back in one copy: the chain summary and every status
    uint8_t *hb = pin + meta_a;
    ZT_TRY(x_copy(hb, d_ust, ust_bytes + st_bytes + sizeof(ChainInfo) + 4, s));
    ZT_HIP(hipStreamSynchronize(s));
    IT("resolved (device chain)");
    const ChainInfo info = *reinterpret_cast<const ChainInfo *>(hb + ust_bytes + st_bytes);
    if (info.ok) {
      if (boundary != ~0ull && !*reinterpret_cast<const uint32_t *>(hb + ust_bytes + st_bytes + sizeof(ChainInfo)))
        FALLBACK("no unit of the chain starts at the boundary %llu\n", (unsigned long long)boundary);
      ZT_TRY(timing_collect(c, &c->times.inflate_ms, &c->times.inflate_launches, 2));
      ZT_TRY(timing_collect(c, &c->times.inflate_tok_ms, &c->times.inflate_toks, 3));
      const int32_t *h_ust = reinterpret_cast<const int32_t *>(hb);
      const int32_t *h_st = reinterpret_cast<const int32_t *>(hb + ust_bytes);
      for (size_t i = 0; i < units; ++i)
        if (h_ust[i] != ZT_OK) FALLBACK("unit %zu of %zu (device chain): status %d\n", i, units, h_ust[i]);
      for (size_t i = 0; i < info.nseg; ++i)
        if (h_st[i] != ZT_OK) FALLBACK("segment %zu of %u: status %d\n", i, info.nseg, h_st[i]);
      *out_len = info.total;
      *end_ip = (info.end_bits + 7) >> 3;
      c->times.inflate_paths[0]++;
      return ZT_OK;
    }
    // not the common case: the host walks the chain (the kernels above did nothing)
    ZT_TRY(timing_begin(c, s, 2));
  }
host_walk:
  TokResult *res = reinterpret_cast<TokResult *>(pin + restart_bytes);
  ZT_TRY(x_copy(pin, d_restart, nsync, s));
  ZT_TRY(x_copy(res, d_res, units * sizeof(TokResult), s));
  const uint64_t *tok_off = reinterpret_cast<const uint64_t *>(pin + restart_bytes + res_bytes);
  ZT_TRY(x_copy(pin + restart_bytes + res_bytes, d_off, units * 8, s));
  ZT_HIP(hipStreamSynchronize(s));
  IT("tokenized");
  if (check) {
    std::vector<uint64_t> dbg(units * 8);
    ZT_HIP(hipMemcpy(dbg.data(), tp.dbg, units * 64, hipMemcpyDeviceToHost));
    size_t bad = 0;
    for (size_t i = 0; i < units; ++i)
      if (dbg[i * 8]) {
        if (bad++ < 8)
          fprintf(stderr, "[zt tok check] unit %zu body@%llu: end simt %llu scalar %llu, tokens %llu/%llu, bytes %llu/%llu\n",
                  i, (unsigned long long)dbg[i * 8 + 1], (unsigned long long)dbg[i * 8 + 2],
                  (unsigned long long)dbg[i * 8 + 3], (unsigned long long)dbg[i * 8 + 4],
                  (unsigned long long)dbg[i * 8 + 5], (unsigned long long)dbg[i * 8 + 6],
                  (unsigned long long)dbg[i * 8 + 7]);
      }
    fprintf(stderr, "[zt tok check] %zu of %zu units differ\n", bad, units);
    if (tp.dump_unit < units) {
      std::vector<uint32_t> dd(8 * 64 * 8);
      ZT_HIP(hipMemcpy(dd.data(), tp.dbg + units * 8, dd.size() * 4, hipMemcpyDeviceToHost));
      for (int r = 0; r < 8; ++r) {
        if (r > 0 && dd[(r * 64) * 8] == 0) break;
        fprintf(stderr, "round %d R=%u last=%d\n", r, dd[(r * 64) * 8], (int)dd[(r * 64) * 8 + 6]);
        for (int l = 0; l < 64; ++l) {
          const uint32_t *d = &dd[(r * 64 + l) * 8];
          fprintf(stderr, "  l%02d t=%u end=%u tok=%u e=%d fl=%u ev=%u\n", l, d[1], d[2], d[3], (int)d[4], d[5], d[7]);
        }
      }
    }
  }
  // 3. the chain from the stream start, cut into segments at restart markers
  std::vector<size_t> chained;  // (units on the chain, for the boundary check)
  std::vector<ChainUnit> chain;
  std::vector<SegJob> segs;
  uint64_t total = 0, seg_start = 0, desc_total = 0, desc_seg = 0;
  size_t u = 0;
  for (;;) {
    const TokResult &r = res[u];
    // the chain reached the last unit (which runs to the end of the input)
    // and that one ran out of input: a window that cuts a longer stream
    // (inflate_dev_member grows it) -- or a truncated stream
    if (u + 1 == units && u > 0 && (r.status == ZT_E_INPUT_BROKEN || r.status == ZT_E_STORED_LEN)) {
      if (inf_debug()) fprintf(stderr, "[zt inflate] chain ran out of input in its last unit %zu\n", u);
      return 2;
    }
    if (r.status != ZT_OK || r.out_len > 0xFFFFFFFFull)
      FALLBACK("unit %zu (chain %zu): status %d detail %d ntok %u out %llu\n", u, chain.size(), r.status,
               r.detail, r.ntok, (unsigned long long)r.out_len);
    // (a restart point right after another -- the empty stored blocks of a
    // restart marker -- leaves the segment before it empty: that one simply
    // starts here instead.  Empty copy waves would sit between the full ones
    // in the launch, and the workgroup -> XCD round robin would then give
    // half of the XCDs every 1 MiB segment: two rounds of copy waves.)
    const bool seg_start_here = u == 0 || restart[u - 1];
    if (segs.empty() || (seg_start_here && total != seg_start)) {
      desc_total = (desc_total + 511) & ~uint64_t(511);
      desc_seg = desc_total;
      seg_start = total;
      segs.push_back(SegJob{(uint32_t)chain.size(), 0});
    }
    chain.push_back(ChainUnit{tok_off[u], total, seg_start, desc_seg + (total - seg_start), r.ntok,
                              (uint32_t)r.out_len});
    chained.push_back(u);
    segs.back().count++;
    total += r.out_len;
    desc_total = desc_seg + (total - seg_start);
    if (r.stop_idx < 0) break;
    const size_t nx = (size_t)r.stop_idx + 1;
    if (nx <= u || nx >= units) FALLBACK("unit %zu: bad stop %d\n", u, r.stop_idx);
    u = nx;
  }
  // a segment of units that hold stored runs only (TokResult ntok bit 30;
  // or nothing) is written by expand_kernel straight from the input and
  // skipped by copy_kernel (SegJob count bit 31); elsewhere bit 30 is cleared
  for (SegJob &sj : segs) {
    bool direct = true;
    for (uint32_t k = 0; k < sj.count; ++k) {
      const ChainUnit &cu = chain[sj.first + k];
      direct = direct && ((cu.ntok >> 30) == 3u || cu.out_len == 0);  // (empty units: the restart markers)
    }
    for (uint32_t k = 0; k < sj.count && !direct; ++k) chain[sj.first + k].ntok &= ~0x40000000u;
    if (direct) sj.count |= 0x80000000u;
  }
  if (boundary != ~0ull) {
    std::vector<TokJob> hj(units);
    ZT_TRY(readback(c, hj.data(), d_jobs, units * sizeof(TokJob), s));
    bool at = false;
    for (size_t k : chained) at = at || hj[k].start == boundary;
    if (!at) FALLBACK("no unit of the chain starts at the boundary %llu\n", (unsigned long long)boundary);
  }
  *out_len = total;
  *end_ip = (res[u].end_bits + 7) >> 3;
  if (inf_debug()) {
    // segment sizes (copy_kernel: one wave per segment)
    uint64_t mn = ~0ull, mx = 0;
    size_t small = 0;
    for (size_t i = 0; i < segs.size(); ++i) {
      const ChainUnit &a = chain[segs[i].first], &b = chain[segs[i].first + (segs[i].count & 0x7FFFFFFFu) - 1];
      const uint64_t len = b.out_off + b.out_len - a.out_off;
      mn = len < mn ? len : mn;
      mx = len > mx ? len : mx;
      small += len < (512u << 10);
    }
    fprintf(stderr, "[zt inflate] %zu units, %zu segments, %llu bytes: segment min %llu max %llu, %zu under 512 KiB\n",
            chain.size(), segs.size(), (unsigned long long)total, (unsigned long long)mn, (unsigned long long)mx, small);
  }
  uint8_t *d_out = *d_out_io;
  if (!d_out) {  // caller wants a library-owned buffer (scratch slot 1)
    void *p;
    ZT_TRY(scratch(c, 1, total ? total : 1, &p));
    d_out = static_cast<uint8_t *>(p);
    *d_out_io = d_out;
  } else if (total > out_cap) {
    *out_len = total;  // (the bytes needed)
    return set_error(ZT_E_ARG, "output capacity too small");
  }
  // 4. expand (one wave per unit) and copy (one wave per segment)
  void *d_chain, *d_desc;
  const size_t chain_bytes = align256(chain.size() * sizeof(ChainUnit));
  const size_t seg_bytes = align256(segs.size() * sizeof(SegJob));
  const size_t ust_bytes = align256(chain.size() * 4);
  ZT_TRY(scratch(c, 7, chain_bytes + seg_bytes + ust_bytes + align256(segs.size() * 4), &d_chain));
  ZT_TRY(scratch(c, 3, (desc_total + 1024) * 2, &d_desc));  // + slack: chunked descriptor reads
  ChainUnit *d_cu = static_cast<ChainUnit *>(d_chain);
  SegJob *d_sj = reinterpret_cast<SegJob *>(static_cast<uint8_t *>(d_chain) + chain_bytes);
  int32_t *d_ust = reinterpret_cast<int32_t *>(static_cast<uint8_t *>(d_chain) + chain_bytes + seg_bytes);
  int32_t *d_st = reinterpret_cast<int32_t *>(static_cast<uint8_t *>(d_chain) + chain_bytes + seg_bytes + ust_bytes);
  ChainUnit *h_cu = reinterpret_cast<ChainUnit *>(pin + meta_a);
  SegJob *h_sj = reinterpret_cast<SegJob *>(pin + meta_a + align256(units_max * sizeof(ChainUnit)));
  int32_t *h_ust = reinterpret_cast<int32_t *>(pin + meta_a + align256(units_max * sizeof(ChainUnit)) +
                                               align256(units_max * sizeof(SegJob)));
  int32_t *h_st = h_ust + align256(units_max * 4) / 4;
  memcpy(h_cu, chain.data(), chain.size() * sizeof(ChainUnit));
  memcpy(h_sj, segs.data(), segs.size() * sizeof(SegJob));
  ZT_TRY(x_copy(d_cu, h_cu, chain.size() * sizeof(ChainUnit), s));
  ZT_TRY(x_copy(d_sj, h_sj, segs.size() * sizeof(SegJob), s));
  ResolveParams rp;
  rp.tokens = static_cast<const uint32_t *>(d_tok);
  rp.units = d_cu;
  rp.segs = d_sj;
  rp.out = d_out;
  rp.desc = static_cast<uint16_t *>(d_desc);
  rp.unit_status = d_ust;
  rp.seg_status = d_st;
  rp.nunits = (uint32_t)chain.size();
  rp.nseg = (uint32_t)segs.size();
  rp.marker = 0;
  rp.in = d_in;
  IT("chain built");
  ZT_TRY(resolve_segments_dev(rp, s));
  ZT_TRY(timing_end(c, s, 2));
  ZT_TRY(x_copy(h_ust, d_ust, chain.size() * 4, s));
  ZT_TRY(x_copy(h_st, d_st, segs.size() * 4, s));
  ZT_HIP(hipStreamSynchronize(s));
  IT("resolved");
  ZT_TRY(timing_collect(c, &c->times.inflate_ms, &c->times.inflate_launches, 2));
  ZT_TRY(timing_collect(c, &c->times.inflate_tok_ms, &c->times.inflate_toks, 3));
  for (size_t i = 0; i < chain.size(); ++i)
    if (h_ust[i] != ZT_OK) FALLBACK("unit %zu of %zu (chain): status %d\n", i, chain.size(), h_ust[i]);
  for (size_t i = 0; i < segs.size(); ++i)
    if (h_st[i] != ZT_OK) FALLBACK("segment %zu of %zu: status %d\n", i, segs.size(), h_st[i]);
  c->times.inflate_paths[0]++;
  return ZT_OK;
}

}  // namespace zt
