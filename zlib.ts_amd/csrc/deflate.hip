// deflate.hip -- raw DEFLATE (RFC 1951) encoder on the GPU.
// Replaces src/LZ77.ts, src/RawDeflate.ts, src/Heap.ts and src/Bitstream.ts.
//
// Geometry (MI355X: 160 KiB LDS per CU, 16 waves):
//   * one 1024-thread workgroup owns a "super-chunk" of K consecutive 32 KiB
//     DEFLATE blocks and streams it through a 36 KiB LDS data ring in 4 KiB
//     sub-chunks, so every position sees the full 32 KiB window (the 32 KiB
//     before the super-chunk is indexed first as history -- halo);
//   * hash chains (13-bit hash of 3 bytes, u16 relative links) live in LDS for
//     the whole ring.  A sub-chunk's links are built lane-parallel: 64-position
//     steps find their in-step predecessors with ballot peer masks, then one
//     wave links the steps to the head table in order (~15 VALU per step);
//   * every position of a sub-chunk searches its chain in parallel (4 positions
//     per thread, newest first, depth-limited, a predecessor's match carried
//     forward one byte), results land in LDS;
//   * one wave parses the sub-chunk 64 positions at a time: next(p) is a
//     function of p (greedy, or one-step lazy), so pointer doubling over
//     v_bpermute finds the parse path in 6 rounds per window; path tokens are
//     compacted with popcount and appended to a per-workgroup token buffer;
//   * at each 32 KiB boundary one wave builds length-limited Huffman codes
//     (bitonic sort + in-place Moffat-Katajainen + JPEG-style limiting), picks
//     the smallest of dynamic / fixed / stored, and all threads encode: prefix
//     sum of per-thread bit counts, interior words stored directly, shared
//     boundary words merged by their first-touching thread.  Every block ends
//     byte-aligned with an empty stored block (00 00 FF FF), so blocks
//     concatenate bytewise (and the stream ends with a final empty stored
//     block, which the reference's over-strict inflate accepts).
#include "zt_internal.h"

namespace zt {

constexpr int DF_BLOCK = 32768;
constexpr int DF_SUB = 4096;
constexpr int DF_RING = DF_BLOCK + DF_SUB;  // 36864 = 9 * 4096
constexpr int DF_SLOT = DF_BLOCK + DF_BLOCK / 8 + 512;  // per-block slot: fits a forced fixed-code block
constexpr int DF_HBITS = 13;
constexpr int DF_THREADS = 1024;
constexpr int DF_MAXDIST = 32768;
// Independent segments of 1 MiB: restart points for segment-parallel inflate
constexpr uint32_t kRestartBlocks = 32;

struct DeflateParams {
  const uint8_t *base;  // stream bytes are base[halo .. halo + n)
  uint64_t halo;
  uint64_t end;         // halo + n
  uint32_t blocks_per_wg;
  uint32_t nblocks;
  uint32_t restart;     // blocks per independent segment (multiple of blocks_per_wg)
  int final_;
  int max_chain;
  int nice_len;
  int lazy;
  int too_far;
  int ctype;            // 1: fixed codes only; 2: best of dynamic/fixed/stored
  uint32_t *tokens;     // nwg x DF_BLOCK
  uint8_t *slots;       // nblocks x DF_SLOT
  uint32_t *slot_len;   // nblocks
  uint32_t *dbg;        // debug dump (first sub-chunk: res[4096], path masks) or null
};

namespace {

__constant__ uint16_t kLenBase[29] = {3,  4,  5,  6,  7,  8,  9,  10, 11,  13,  15,  17,  19,  23, 27,
                                      31, 35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 258};
__constant__ uint8_t kLenExtra[29] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2,
                                      2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
__constant__ uint8_t kClOrder[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

struct EncScratch {
  uint32_t start[DF_THREADS + 1];  // exclusive prefix of per-thread bit counts
  uint32_t first_val[DF_THREADS];  // contribution to the (partial) first word
  uint32_t sizes[4];
};

struct HufScratch {
  uint32_t key[512];  // (freq << 9) | symbol, sorted ascending
  uint32_t a[320];    // Moffat-Katajainen work array
  uint32_t bl_count[40];
};

struct DefShared {
  uint32_t ring[DF_RING / 4 + 16];  // data ring + 64-byte mirror of its start
  uint16_t prev[DF_RING];           // relative chain links (0 = none)
  uint16_t head[1 << DF_HBITS];     // last position (mod 65536) per hash
  union {
    uint32_t res[DF_SUB];           // per-position match: len << 16 | dist
    EncScratch enc;
    HufScratch huf;
  } u;
  uint32_t lit_hist[288];
  uint32_t dist_hist[32];
  uint32_t lit_code[288];   // len << 16 | bit-reversed code
  uint32_t dist_code[32];
  uint32_t cl_code[19];
  uint8_t lit_len[288];
  uint8_t dist_len[32];
  uint8_t cl_len[19];
  uint16_t cl_syms[320];    // sym | extra_value << 5
  uint32_t n_cl_syms, hlit, hdist, hclen;
  uint32_t ntok;
  uint32_t btype;           // chosen block type: 0 stored, 1 fixed, 2 dynamic
  uint32_t hdr_bits;
};

// ---- ring addressing ---------------------------------------------------------
__device__ __forceinline__ uint32_t ridx(uint32_t rel) {
  uint32_t q = __umulhi(rel >> 12, 0x1C71C71Du);  // (rel >> 12) / 9, exact for rel < 2^31
  return rel - q * (uint32_t)DF_RING;
}
__device__ __forceinline__ uint32_t ld8(const DefShared *s, uint32_t rel) {
  return reinterpret_cast<const uint8_t *>(s->ring)[ridx(rel)];
}
__device__ __forceinline__ uint32_t ld32(const DefShared *s, uint32_t rel) {
  uint32_t i = ridx(rel);
  uint32_t w = i >> 2;
  return __builtin_amdgcn_alignbyte(s->ring[w + 1], s->ring[w], i & 3);
}
// chains link positions whose first DF_MINH (3 or 4) bytes hash alike
#ifndef DF_MINH
#define DF_MINH 3
#endif
constexpr uint32_t kKeyMask = DF_MINH >= 4 ? 0xFFFFFFFFu : 0xFFFFFFu;
__device__ __forceinline__ uint32_t hash3(uint32_t v) { return ((v & kKeyMask) * 0x9E3779B1u) >> (32 - DF_HBITS); }

__device__ __forceinline__ uint64_t lanemask_lt(int lane) { return lane ? (~0ull >> (64 - lane)) : 0ull; }

__device__ __forceinline__ uint32_t dist_sym(uint32_t d, uint32_t &ebits, uint32_t &evalue) {
  if (d <= 4) {
    ebits = 0;
    evalue = 0;
    return d - 1;
  }
  uint32_t x = d - 1;
  uint32_t k = 31 - __clz(x);
  ebits = k - 1;
  evalue = x & ((1u << (k - 1)) - 1);
  return 2 * k + ((x >> (k - 1)) & 1);
}

__device__ __forceinline__ uint32_t len_sym(uint32_t L) {
  // index into kLenBase (0..28)
  if (L == 258) return 28;
  if (L <= 10) return L - 3;
  uint32_t x = L - 3;
  uint32_t k = 31 - __clz(x);  // >= 3
  return 4 * (k - 1) + ((x >> (k - 2)) & 3);
}

// ---- phase: load a sub-chunk's bytes into the ring ----------------------------------
__device__ void load_sub(DefShared *s, const uint8_t *g, uint32_t rel0, uint32_t len) {
  uint8_t *rb = reinterpret_cast<uint8_t *>(s->ring);
  for (uint32_t i = threadIdx.x; i < len; i += DF_THREADS) {
    uint8_t v = g[i];
    uint32_t k = ridx(rel0 + i);
    rb[k] = v;
    if (k < 64) rb[DF_RING + k] = v;
  }
}

// ---- phase: chain links for positions [lo, hi) (rel coords) ---------------------------
__device__ void chain_build(DefShared *s, uint32_t lo, uint32_t hi) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint32_t nsteps = (hi - lo + 63) / 64;
  // (1) in-step predecessors, all waves
  for (uint32_t st = wave; st < nsteps; st += DF_THREADS / 64) {
    uint32_t p = lo + st * 64 + lane;
    bool valid = p < hi;
    uint32_t h = valid ? hash3(ld32(s, p)) : 0;
    uint64_t peers = __ballot(valid);
#pragma unroll
    for (int b = 0; b < DF_HBITS; ++b) {
      uint64_t m = __ballot((h >> b) & 1);
      peers &= ((h >> b) & 1) ? m : ~m;
    }
    uint64_t below = peers & lanemask_lt(lane);
    uint64_t above = peers & ~((2ull << lane) - 1);
    uint32_t d = below ? (uint32_t)(lane - (63 - __clzll(below))) : 0u;
    if (valid) s->prev[ridx(p)] = (uint16_t)(d | (above ? 0 : 0x8000));
  }
  __syncthreads();
  // (2) one wave links steps to the head table in position order
  if (wave == 0) {
    for (uint32_t st = 0; st < nsteps; ++st) {
      uint32_t p = lo + st * 64 + lane;
      bool valid = p < hi;
      uint32_t h = 0, e = 0, hv = 0;
      if (valid) {
        e = s->prev[ridx(p)];
        h = hash3(ld32(s, p));
        hv = s->head[h];
      }
      uint32_t link = e & 0x7F;
      if (valid && link == 0) {
        uint32_t d = (p - hv) & 0xFFFF;
        // reject stale head entries: the linked position must carry the same hash
        if (d == 0 || d > DF_MAXDIST || d > p || hash3(ld32(s, p - d)) != h) d = 0;
        link = d;
      }
      if (valid) {
        s->prev[ridx(p)] = (uint16_t)link;
        if (e & 0x8000) s->head[h] = (uint16_t)(p & 0xFFFF);
      }
    }
  }
  __syncthreads();
}

// ---- phase: per-position longest-match search ------------------------------------------
__device__ void search_sub(DefShared *s, const DeflateParams &P, uint32_t p0, uint32_t p1, uint32_t lo_bound) {
  const uint32_t t = threadIdx.x;
  uint32_t carry_len = 0, carry_dist = 0;
#pragma unroll 1
  for (int k = 0; k < 4; ++k) {
    const uint32_t p = p0 + t * 4 + k;
    if (p >= p1) break;
    const uint32_t max_len = (p1 - p) < 258 ? (p1 - p) : 258;
    uint32_t best_len = 0, best_dist = 0;
    if (max_len >= 3) {
      if (carry_len > 3) {
        best_len = carry_len - 1;
        best_dist = carry_dist;
      }
      if ((int)best_len < P.nice_len) {
        const uint32_t cur = ld32(s, p);
        uint32_t link = s->prev[ridx(p)];
        uint32_t q = p;
        int hops = 0;
#pragma unroll 1
        while (link && hops < P.max_chain) {
          q -= link;
          if (p - q > DF_MAXDIST || q < lo_bound) break;
          ++hops;
          link = s->prev[ridx(q)];
          if (((ld32(s, q) ^ cur) & kKeyMask) != 0) continue;
          if (best_len >= max_len) break;
          if (best_len >= 4) {
            // a candidate can only beat best_len if the 4 bytes ending there match
            const uint32_t o = best_len - 3;
            if (ld32(s, q + o) != ld32(s, p + o)) continue;
          }
          uint32_t len = DF_MINH;
          while (len < max_len) {
            uint32_t x = ld32(s, q + len) ^ ld32(s, p + len);
            if (x) {
              len += (uint32_t)(__ffs(x) - 1) >> 3;
              break;
            }
            len += 4;
          }
          if (len > max_len) len = max_len;
          if (len > best_len) {
            best_len = len;
            best_dist = p - q;
            if ((int)len >= P.nice_len) break;
          }
        }
      }
    }
    carry_len = best_len;
    carry_dist = best_dist;
    if (best_len == 3 && best_dist > (uint32_t)P.too_far) best_len = 0;
    s->u.res[p - p0] = best_len >= 3 ? (best_len << 16) | best_dist : 0u;
  }
}

// ---- phase: parse a sub-chunk (wave 0) --------------------------------------------------
__device__ void parse_sub(DefShared *s, const DeflateParams &P, uint32_t p0, uint32_t p1, uint32_t *tok) {
  const int lane = threadIdx.x & 63;
  const uint32_t len = p1 - p0;
  uint32_t entry = 0;  // first path position relative to the current window
  uint32_t ntok = s->ntok;
  for (uint32_t w0 = 0; w0 < len; w0 += 64) {
    if (entry >= 64) {
      entry -= 64;
      continue;
    }
    const uint32_t i = w0 + lane;
    uint32_t r = i < len ? s->u.res[i] : 0u;
    uint32_t L = r >> 16;
    if (L >= 3 && P.lazy && i + 1 < len) {
      uint32_t L2 = s->u.res[i + 1] >> 16;
      if (L2 > L) L = 0;
    }
    const uint32_t step = L >= 3 ? L : 1;
    // positions past the sub-chunk end terminate the path without emitting
    uint32_t ptr = i < len ? lane + step : 64u;  // relative to the window start
    uint64_t mask = i < len ? 1ull << lane : 0ull;
#pragma unroll
    for (int rnd = 0; rnd < 6; ++rnd) {
      const bool in = ptr < 64;
      const int src = in ? (int)ptr : lane;
      uint32_t mlo = __shfl((uint32_t)mask, src, 64);
      uint32_t mhi = __shfl((uint32_t)(mask >> 32), src, 64);
      uint32_t nptr = __shfl(ptr, src, 64);
      if (in) {
        mask |= ((uint64_t)mhi << 32) | mlo;
        ptr = nptr;
      }
    }
    // (readlane returns int: go through uint32_t so the low half is not sign-extended)
    const uint32_t path_hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(mask >> 32), (int)entry);
    const uint32_t path_lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)mask, (int)entry);
    const uint64_t path = ((uint64_t)path_hi << 32) | path_lo;
    const uint32_t exit = (uint32_t)__builtin_amdgcn_readlane((int)ptr, (int)entry);
    const bool on = (path >> lane) & 1;
    if (P.dbg && p0 == 0 && blockIdx.x == 0) {
      P.dbg[i] = r;
      P.dbg[4096 + i] = ptr;
      P.dbg[8192 + i] = (uint32_t)mask;
      P.dbg[12288 + i] = (uint32_t)(mask >> 32);
      if (lane == 0) P.dbg[16384 + w0 / 64] = entry;
    }
    if (on) {
      uint32_t token;
      if (L >= 3) {
        token = (L << 16) | (r & 0xFFFF);
        uint32_t eb, ev;
        atomicAdd(&s->lit_hist[257 + len_sym(L)], 1u);
        atomicAdd(&s->dist_hist[dist_sym(r & 0xFFFF, eb, ev)], 1u);
      } else {
        token = ld8(s, p0 + i);
        atomicAdd(&s->lit_hist[token], 1u);
      }
      tok[ntok + __popcll(path & lanemask_lt(lane))] = token;
    }
    ntok += __popcll(path);
    entry = exit - 64;
  }
  if (lane == 0) s->ntok = ntok;
}

// ---- Huffman code lengths (one wave) -------------------------------------------------------
// freq[0..n) -> len[0..n), limited to `limit` bits.  Always produces a complete
// code with >= 2 symbols (zlib's rule), forcing symbols 0/1 in when needed.
__device__ void huff_lengths(DefShared *s, const uint32_t *freq_in, int n, int limit, uint8_t *len_out) {
  const int lane = threadIdx.x & 63;
  HufScratch &h = s->u.huf;
  // keys for all symbols; absent symbols sort last
  for (int i = lane; i < 512; i += 64) {
    uint32_t f = i < n ? freq_in[i] : 0;
    h.key[i] = (i < n && f) ? ((f << 9) | (uint32_t)i) : 0xFFFFFFFFu;
  }
  for (int i = lane; i < n; i += 64) len_out[i] = 0;
  // (wave-0-only code: LDS ops of one wave complete in order; the fences only
  // keep the compiler from reordering.  No s_barrier here -- the other waves
  // are parked at the caller's __syncthreads().)
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
  // count present symbols
  uint32_t m = 0;
  for (int i = lane; i < n; i += 64) m += (freq_in[i] != 0);
  for (int off = 32; off; off >>= 1) m += __shfl_xor(m, off, 64);
  if (m < 2) {
    // force a second symbol so that the code is complete (RFC 1951 decoders
    // such as zlib reject a single one-bit code set for lit/len)
    if (lane == 0) {
      int a = -1;
      for (int i = 0; i < n; ++i)
        if (freq_in[i]) a = i;
      int b0 = (a == 0) ? 1 : 0;
      if (a < 0) {
        len_out[0] = 1;
        len_out[1] = 1;
      } else {
        len_out[a] = 1;
        len_out[b0] = 1;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
    return;
  }
  // bitonic sort of 512 keys, ascending
  for (int k = 2; k <= 512; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = lane; i < 512; i += 64) {
        int ixj = i ^ j;
        if (ixj > i) {
          uint32_t a = h.key[i], b = h.key[ixj];
          bool up = (i & k) == 0;
          if ((a > b) == up) {
            h.key[i] = b;
            h.key[ixj] = a;
          }
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
    }
  }
  if (lane == 0) {
    uint32_t *A = h.a;
    for (uint32_t i = 0; i < m; ++i) A[i] = h.key[i] >> 9;
    // Moffat & Katajainen, in-place minimum-redundancy code lengths
    int mm = (int)m;
    int sidx = 0, r = 0;
    for (int t = 0; t < mm - 1; ++t) {
      if (sidx >= mm || (r < t && A[r] < A[sidx])) {
        A[t] = A[r];
        A[r] = t;
        ++r;
      } else {
        A[t] = A[sidx];
        ++sidx;
      }
      if (sidx >= mm || (r < t && A[r] < A[sidx])) {
        A[t] += A[r];
        A[r] = t;
        ++r;
      } else {
        A[t] += A[sidx];
        ++sidx;
      }
    }
    A[mm - 2] = 0;
    for (int t = mm - 3; t >= 0; --t) A[t] = A[A[t]] + 1;
    int avail = 1, used = 0, depth = 0, t = mm - 2, x = mm - 1;
    while (avail > 0) {
      while (t >= 0 && (int)A[t] == depth) {
        ++used;
        --t;
      }
      while (avail > used) {
        A[x] = depth;
        --x;
        --avail;
      }
      avail = 2 * used;
      ++depth;
      used = 0;
    }
    // A[i] = length of the i-th least frequent symbol; limit via bl_count
    uint32_t *bl = h.bl_count;
    for (int i = 0; i < 40; ++i) bl[i] = 0;
    int maxl = 0;
    for (int i = 0; i < mm; ++i) {
      int l = (int)A[i];
      if (l > 39) l = 39;
      bl[l]++;
      if (l > maxl) maxl = l;
    }
    for (int i = maxl; i > limit; --i) {
      while (bl[i] > 0) {
        int j = i - 2;
        while (bl[j] == 0) --j;
        bl[i] -= 2;
        bl[i - 1] += 1;
        bl[j + 1] += 2;
        bl[j] -= 1;
      }
    }
    // longest codes go to the least frequent symbols
    int l = limit < maxl ? limit : maxl;
    int idx = 0;
    for (; l >= 1; --l)
      for (uint32_t c = 0; c < bl[l]; ++c) len_out[h.key[idx++] & 511] = (uint8_t)l;
  }
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
}

// canonical codes (bit-reversed for LSB-first emission), one wave
__device__ void huff_codes(const uint8_t *len, int n, uint32_t *code) {
  const int lane = threadIdx.x & 63;
  if (lane == 0) {
    uint32_t cnt[16] = {0}, next[16];
    for (int i = 0; i < n; ++i) cnt[len[i]]++;
    cnt[0] = 0;
    uint32_t c = 0;
    for (int l = 1; l < 16; ++l) {
      c = (c + cnt[l - 1]) << 1;
      next[l] = c;
    }
    for (int i = 0; i < n; ++i) {
      uint32_t l = len[i];
      if (!l) {
        code[i] = 0;
        continue;
      }
      uint32_t v = next[l]++;
      code[i] = (l << 16) | (__brev(v) >> (32 - l));
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
}

__device__ __forceinline__ uint32_t fixed_lit(uint32_t sym) {
  uint32_t l, c;
  if (sym <= 143) {
    l = 8;
    c = 0x30 + sym;
  } else if (sym <= 255) {
    l = 9;
    c = 0x190 + sym - 144;
  } else if (sym <= 279) {
    l = 7;
    c = sym - 256;
  } else {
    l = 8;
    c = 0xC0 + sym - 280;
  }
  return (l << 16) | (__brev(c) >> (32 - l));
}

// ---- block header (one wave): codes, RLE of lengths, choice of block type ----------------------
__device__ void plan_block(DefShared *s, const DeflateParams &P, uint32_t blen) {
  const int lane = threadIdx.x & 63;
  if (lane == 0) s->lit_hist[256] += 1;  // end of block
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
  huff_lengths(s, s->lit_hist, 286, 15, s->lit_len);
  huff_lengths(s, s->dist_hist, 30, 15, s->dist_len);
  if (lane == 0) {
    uint32_t hlit = 286, hdist = 30;
    while (hlit > 257 && s->lit_len[hlit - 1] == 0) --hlit;
    while (hdist > 1 && s->dist_len[hdist - 1] == 0) --hdist;
    s->hlit = hlit;
    s->hdist = hdist;
    // RLE of the concatenated lengths (RFC 1951 3.2.7)
    uint32_t nsym = 0;
    const uint32_t total = hlit + hdist;
    uint32_t clf[19] = {0};
    uint32_t i = 0;
    while (i < total) {
      uint32_t v = i < hlit ? s->lit_len[i] : s->dist_len[i - hlit];
      uint32_t run = 1;
      while (i + run < total && (i + run < hlit ? s->lit_len[i + run] : s->dist_len[i + run - hlit]) == v) ++run;
      i += run;
      if (v == 0) {
        while (run >= 11) {
          uint32_t r = run < 138 ? run : 138;
          s->cl_syms[nsym++] = 18 | ((r - 11) << 5);
          clf[18]++;
          run -= r;
        }
        if (run >= 3) {
          s->cl_syms[nsym++] = 17 | ((run - 3) << 5);
          clf[17]++;
          run = 0;
        }
        while (run--) {
          s->cl_syms[nsym++] = 0;
          clf[0]++;
        }
      } else {
        s->cl_syms[nsym++] = v;
        clf[v]++;
        --run;
        while (run >= 3) {
          uint32_t r = run < 6 ? run : 6;
          s->cl_syms[nsym++] = 16 | ((r - 3) << 5);
          clf[16]++;
          run -= r;
        }
        while (run--) {
          s->cl_syms[nsym++] = v;
          clf[v]++;
        }
      }
    }
    s->n_cl_syms = nsym;
    // cl_code[] doubles as the CL symbol frequencies until the codes are built
    for (int k = 0; k < 19; ++k) s->cl_code[k] = clf[k];
  }
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
  huff_lengths(s, s->cl_code, 19, 7, s->cl_len);
  huff_codes(s->lit_len, 286, s->lit_code);
  huff_codes(s->dist_len, 30, s->dist_code);
  huff_codes(s->cl_len, 19, s->cl_code);
  // sizes of the three choices (bits, without the sync marker)
  uint64_t dyn = 0, fix = 0;
  for (int i = lane; i < 286; i += 64) {
    uint32_t f = s->lit_hist[i];
    uint32_t extra = i >= 257 ? kLenExtra[i - 257] : 0;
    dyn += (uint64_t)f * (s->lit_len[i] + extra);
    fix += (uint64_t)f * ((fixed_lit(i) >> 16) + extra);
  }
  if (lane < 30) {
    uint32_t f = s->dist_hist[lane];
    uint32_t extra = lane < 4 ? 0 : (lane >> 1) - 1;
    dyn += (uint64_t)f * (s->dist_len[lane] + extra);
    fix += (uint64_t)f * (5 + extra);
  }
  for (int off = 32; off; off >>= 1) {
    dyn += __shfl_xor(dyn, off, 64);
    fix += __shfl_xor(fix, off, 64);
  }
  if (lane == 0) {
    uint32_t hclen = 19;
    while (hclen > 4 && s->cl_len[kClOrder[hclen - 1]] == 0) --hclen;
    s->hclen = hclen;
    uint32_t hdr = 3 + 5 + 5 + 4 + 3 * hclen;
    for (uint32_t k = 0; k < s->n_cl_syms; ++k) {
      uint32_t c = s->cl_syms[k] & 31;
      hdr += s->cl_len[c] + (c == 16 ? 2 : c == 17 ? 3 : c == 18 ? 7 : 0);
    }
    dyn += hdr;
    fix += 3;
    // stored: this block's bytes + 5 header bytes; Huffman forms add the
    // 3-bit marker header, padding and the 4 sync bytes
    uint64_t stored_bits = 8ull * (blen + 5);
    uint64_t dyn_bits = ((dyn + 3 + 7) & ~7ull) + 32;
    uint64_t fix_bits = ((fix + 3 + 7) & ~7ull) + 32;
    uint32_t bt;
    if (P.ctype == 1) bt = 1;
    else if (stored_bits <= dyn_bits && stored_bits <= fix_bits) bt = 0;
    else bt = dyn_bits <= fix_bits ? 2 : 1;
    s->btype = bt;
    s->hdr_bits = bt == 2 ? hdr : 3;
  }
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
}

// bit accumulator writing aligned 32-bit words of one block slot
struct BitOut {
  uint64_t acc;
  uint32_t nacc;      // valid bits in acc (acc bit 0 = bit `word * 32` of the block)
  uint32_t word;      // index of the word acc starts at
  uint32_t first;     // first word index of this thread's range
  uint32_t *slot;
  uint32_t first_val;
  bool first_partial;
  bool wrote_first;

  __device__ void init(uint32_t start_bit, uint32_t *sl) {
    slot = sl;
    word = start_bit >> 5;
    first = word;
    nacc = start_bit & 31;
    acc = 0;
    first_partial = nacc != 0;
    wrote_first = false;
    first_val = 0;
  }
  __device__ __forceinline__ void put(uint32_t v, uint32_t n) {
    acc |= (uint64_t)v << nacc;
    nacc += n;
    if (nacc >= 32) {
      uint32_t w = (uint32_t)acc;
      if (word == first && first_partial) {
        first_val = w;
        wrote_first = true;
      } else {
        slot[word] = w;
      }
      ++word;
      acc >>= 32;
      nacc -= 32;
    }
  }
};

__device__ __forceinline__ void put_token(BitOut &bo, const DefShared *s, uint32_t tk, bool fixed) {
  if (tk < 256) {
    uint32_t c = fixed ? fixed_lit(tk) : s->lit_code[tk];
    bo.put(c & 0xFFFF, c >> 16);
    return;
  }
  uint32_t L = tk >> 16, D = tk & 0xFFFF;
  uint32_t ls = len_sym(L);
  uint32_t c = fixed ? fixed_lit(257 + ls) : s->lit_code[257 + ls];
  bo.put(c & 0xFFFF, c >> 16);
  if (kLenExtra[ls]) bo.put(L - kLenBase[ls], kLenExtra[ls]);
  uint32_t eb, ev;
  uint32_t ds = dist_sym(D, eb, ev);
  if (fixed) {
    bo.put(__brev(ds) >> 27, 5);
  } else {
    uint32_t dc = s->dist_code[ds];
    bo.put(dc & 0xFFFF, dc >> 16);
  }
  if (eb) bo.put(ev, eb);
}

__device__ __forceinline__ uint32_t token_bits(const DefShared *s, uint32_t tk, bool fixed) {
  if (tk < 256) return fixed ? (fixed_lit(tk) >> 16) : s->lit_len[tk];
  uint32_t L = tk >> 16, D = tk & 0xFFFF;
  uint32_t ls = len_sym(L);
  uint32_t eb, ev;
  uint32_t ds = dist_sym(D, eb, ev);
  return (fixed ? (fixed_lit(257 + ls) >> 16) : s->lit_len[257 + ls]) + kLenExtra[ls] +
         (fixed ? 5u : s->dist_len[ds]) + eb;
}

// ---- encode the block (all threads) -------------------------------------------------------
__device__ void encode_block(DefShared *s, const DeflateParams &P, const uint32_t *tok, uint32_t ntok,
                             uint8_t *slot_bytes, uint32_t *slot_len, const uint8_t *raw, uint32_t blen,
                             bool last) {
  const uint32_t t = threadIdx.x;
  const uint32_t bt = s->btype;
  if (bt == 0) {
    // stored block: header byte, LEN, NLEN, data
    if (t == 0) {
      slot_bytes[0] = last ? 1 : 0;
      slot_bytes[1] = blen & 0xFF;
      slot_bytes[2] = blen >> 8;
      slot_bytes[3] = (~blen) & 0xFF;
      slot_bytes[4] = ((~blen) >> 8) & 0xFF;
      *slot_len = blen + 5;
    }
    for (uint32_t i = t; i < blen; i += DF_THREADS) slot_bytes[5 + i] = raw[i];
    __syncthreads();
    return;
  }
  const bool fixed = bt == 1;
  const uint32_t a = (uint32_t)(((uint64_t)ntok * t) / DF_THREADS);
  const uint32_t b = (uint32_t)(((uint64_t)ntok * (t + 1)) / DF_THREADS);
  uint32_t bits = 0;
  for (uint32_t i = a; i < b; ++i) bits += token_bits(s, tok[i], fixed);
  if (t == 0) bits += s->hdr_bits;
  const uint32_t eob = fixed ? (fixed_lit(256) >> 16) : s->lit_len[256];
  if (t == DF_THREADS - 1) bits += eob;  // marker bits appended after the scan
  // exclusive scan over threads (wave shuffles + LDS)
  EncScratch &e = s->u.enc;
  {
    const int lane = t & 63, wave = t >> 6;
    uint32_t x = bits;
    for (int off = 1; off < 64; off <<= 1) {
      uint32_t y = __shfl_up(x, off, 64);
      if (lane >= off) x += y;
    }
    __shared__ uint32_t wsum[16];
    if (lane == 63) wsum[wave] = x;
    __syncthreads();
    if (t < 16) {
      uint32_t v = wsum[t];
      for (int off = 1; off < 16; off <<= 1) {
        uint32_t y = __shfl_up(v, off, 16);
        if ((int)t >= off) v += y;
      }
      wsum[t] = v;
    }
    __syncthreads();
    uint32_t incl = x + (wave ? wsum[wave - 1] : 0);
    e.start[t] = incl - bits;
    if (t == DF_THREADS - 1) e.start[DF_THREADS] = incl;
  }
  __syncthreads();
  uint32_t *slot = reinterpret_cast<uint32_t *>(slot_bytes);
  const uint32_t start = e.start[t];
  uint32_t end = e.start[t + 1];
  uint32_t total_end = e.start[DF_THREADS];
  // marker: 3-bit stored header (BFINAL on the stream's last block), pad, 00 00 FF FF
  const uint32_t after = total_end + 3;
  const uint32_t padded = (after + 7) & ~7u;
  const uint32_t block_end = padded + 32;
  BitOut bo;
  bo.init(start, slot);
  if (t == 0) {
    if (fixed) {
      bo.put(2, 3);  // BFINAL=0, BTYPE=01
    } else {
      bo.put(4, 3);  // BFINAL=0, BTYPE=10
      bo.put(s->hlit - 257, 5);
      bo.put(s->hdist - 1, 5);
      bo.put(s->hclen - 4, 4);
      for (uint32_t k = 0; k < s->hclen; ++k) bo.put(s->cl_len[kClOrder[k]], 3);
      for (uint32_t k = 0; k < s->n_cl_syms; ++k) {
        uint32_t cs = s->cl_syms[k], c = cs & 31;
        uint32_t cc = s->cl_code[c];
        bo.put(cc & 0xFFFF, cc >> 16);
        if (c == 16) bo.put(cs >> 5, 2);
        else if (c == 17) bo.put(cs >> 5, 3);
        else if (c == 18) bo.put(cs >> 5, 7);
      }
    }
  }
  for (uint32_t i = a; i < b; ++i) put_token(bo, s, tok[i], fixed);
  if (t == DF_THREADS - 1) {
    uint32_t c = fixed ? fixed_lit(256) : s->lit_code[256];
    bo.put(c & 0xFFFF, c >> 16);
    bo.put(last ? 1 : 0, 3);
    bo.put(0, padded - after);
    bo.put(0xFFFF0000u, 32);
    end = block_end;
    total_end = block_end;
  }
  // share the partial first word; the first thread touching a word writes it
  e.first_val[t] = bo.first_partial ? (bo.wrote_first ? bo.first_val : (uint32_t)bo.acc) : 0;
  __syncthreads();
  const bool have_tail = bo.nacc > 0 && !(bo.word == bo.first && bo.first_partial);
  if (have_tail) {
    // this thread started at or before the tail word's first bit: it owns it
    const uint32_t w = bo.word;
    uint32_t v = (uint32_t)bo.acc;
    for (uint32_t u = t + 1; u < DF_THREADS; ++u) {
      uint32_t us = e.start[u], ue = (u == DF_THREADS - 1) ? block_end : e.start[u + 1];
      if (ue == us) continue;
      if ((us >> 5) != w) break;
      v |= e.first_val[u];
      if (ue >= (w + 1) * 32) break;
    }
    slot[w] = v;
  }
  (void)end;
  if (t == 0) *slot_len = block_end >> 3;
  __syncthreads();
}

#ifdef ZT_DF_PROF
__device__ unsigned long long g_df_prof[8];
#define DFP_T() ((uint64_t)__builtin_readcyclecounter())
#define DFP_MARK(i)                    \
  do {                                 \
    const uint64_t now_ = DFP_T();     \
    prof[i] += now_ - prof_t;          \
    prof_t = now_;                     \
  } while (0)
#else
#define DFP_MARK(i) ((void)0)
#endif

__global__ __launch_bounds__(DF_THREADS) void deflate_kernel(DeflateParams P) {
  __shared__ DefShared s;
#ifdef ZT_DF_PROF
  uint64_t prof[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  uint64_t prof_t = DFP_T();
#endif
  const uint32_t t = threadIdx.x;
  const uint32_t wg = blockIdx.x;
  const uint32_t b0 = wg * P.blocks_per_wg;
  const uint32_t b1 = (b0 + P.blocks_per_wg) < P.nblocks ? (b0 + P.blocks_per_wg) : P.nblocks;
  const uint64_t s_lo = P.halo + (uint64_t)b0 * DF_BLOCK;
  const uint64_t s_hi = (P.halo + (uint64_t)b1 * DF_BLOCK) < P.end ? (P.halo + (uint64_t)b1 * DF_BLOCK) : P.end;
  // a segment start (restart point) sees no history: its matches stay inside
  // the segment, so inflate can decode segments independently
  const bool restart = (b0 % P.restart) == 0 && (b0 > 0 || P.halo == 0);
  const uint64_t h_lo = restart ? s_lo : (s_lo > DF_MAXDIST ? s_lo - DF_MAXDIST : 0);
  const uint8_t *g = P.base + h_lo;  // rel 0
  const uint32_t rs = (uint32_t)(s_lo - h_lo), re = (uint32_t)(s_hi - h_lo);
  const uint32_t rend = (uint32_t)(P.end - h_lo);  // bytes available (for hashing)
  uint32_t *tok = P.tokens + (size_t)wg * DF_BLOCK;

  for (uint32_t i = t; i < (1u << DF_HBITS); i += DF_THREADS) s.head[i] = (uint16_t)((0u - 40000u) & 0xFFFF);
  for (uint32_t i = t; i < 288; i += DF_THREADS) s.lit_hist[i] = 0;
  if (t < 32) s.dist_hist[t] = 0;
  if (t == 0) s.ntok = 0;
  __syncthreads();

  // history (halo): index [0, rs) without searching
  uint32_t inserted = 0;  // positions [0, inserted) are in the chains
  for (uint32_t p0 = 0; p0 < rs; p0 += DF_SUB) {
    uint32_t p1 = (p0 + DF_SUB) < rs ? (p0 + DF_SUB) : rs;
    load_sub(&s, g + p0, p0, p1 - p0);
    __syncthreads();
    uint32_t ih = p1 >= 2 ? p1 - 2 : 0;
    if (ih > inserted) {
      chain_build(&s, inserted, ih);
      inserted = ih;
    }
  }
  // the super-chunk, 4 KiB at a time
  uint32_t blk = b0;
  uint32_t blk_lo = rs;
  for (uint32_t p0 = rs; p0 < re; p0 += DF_SUB) {
    const uint32_t p1 = (p0 + DF_SUB) < re ? (p0 + DF_SUB) : re;
    load_sub(&s, g + p0, p0, p1 - p0);
    __syncthreads();
    uint32_t ih = p1 - 2 < rend - 2 ? p1 - 2 : rend - 2;
    if (p1 < 2) ih = 0;
    DFP_MARK(0);
    if (ih > inserted) {
      chain_build(&s, inserted, ih);
      inserted = ih;
    }
    DFP_MARK(1);
    search_sub(&s, P, p0, p1, 0);
    __syncthreads();
    DFP_MARK(2);
    if (t < 64) parse_sub(&s, P, p0, p1, tok);
    __syncthreads();
    DFP_MARK(3);
    if (p1 - blk_lo == DF_BLOCK || p1 == re) {
      // finish block `blk` covering [blk_lo, p1)
      const uint32_t blen = p1 - blk_lo;
      const bool last = P.final_ && (blk == P.nblocks - 1);
      if (t < 64) plan_block(&s, P, blen);
      __syncthreads();
      __threadfence_block();
      DFP_MARK(4);
      encode_block(&s, P, tok, s.ntok, P.slots + (size_t)blk * DF_SLOT, P.slot_len + blk, g + blk_lo, blen, last);
      DFP_MARK(5);
      for (uint32_t i = t; i < 288; i += DF_THREADS) s.lit_hist[i] = 0;
      if (t < 32) s.dist_hist[t] = 0;
      if (t == 0) s.ntok = 0;
      __syncthreads();
      ++blk;
      blk_lo = p1;
    }
  }
#ifdef ZT_DF_PROF
  if (t == 0)
    for (int i = 0; i < 8; ++i) atomicAdd(&g_df_prof[i], (unsigned long long)prof[i]);
#endif
}

// ---- stitching: exclusive scan of block sizes, then a byte-exact gather ---------------------------
// A restart point (segment boundary) is announced by two empty stored blocks
// after the preceding block (which always ends byte-aligned):
//   00 00 00 FF FF 00 00 00 FF FF
// An ordinary block boundary carries at most one, so the 10-byte pattern at a
// stored-block end marks a segment that inflate may decode on its own.
constexpr uint32_t kRestartMarkerLen = 10;
// (a non-final call -- a shard -- also ends with the marker: the next shard
// is independent when deflated with halo 0, see zt_shard.py)
__device__ __forceinline__ bool restart_after(uint32_t b, uint32_t n, uint32_t restart, int final_) {
  return (b + 1 < n) ? ((b + 1) % restart) == 0 : !final_;
}

__global__ __launch_bounds__(1024) void scan_sizes(const uint32_t *__restrict__ len, uint32_t n,
                                                   uint64_t *__restrict__ off, uint64_t base, uint32_t restart,
                                                   int final_) {
  __shared__ uint64_t part[1024];
  const uint32_t t = threadIdx.x;
  const uint32_t per = (n + 1023) / 1024;
  const uint32_t a = t * per, b = (a + per) < n ? (a + per) : n;
  uint64_t sum = 0;
  for (uint32_t i = a; i < b; ++i) sum += len[i] + (restart_after(i, n, restart, final_) ? kRestartMarkerLen : 0);
  part[t] = sum;
  __syncthreads();
  for (int d = 1; d < 1024; d <<= 1) {
    uint64_t v = (int)t >= d ? part[t - d] : 0;
    __syncthreads();
    part[t] += v;
    __syncthreads();
  }
  uint64_t run = base + part[t] - sum;
  for (uint32_t i = a; i < b; ++i) {
    off[i] = run;
    run += len[i] + (restart_after(i, n, restart, final_) ? kRestartMarkerLen : 0);
  }
  if (t == 1023) off[n] = base + part[1023];
}

__global__ __launch_bounds__(256) void gather_blocks(const uint8_t *__restrict__ slots, const uint32_t *__restrict__ len,
                                                     const uint64_t *__restrict__ off, uint8_t *__restrict__ out,
                                                     uint32_t nblocks, uint32_t restart, int final_) {
  const uint32_t b = blockIdx.x;
  const uint8_t *src = slots + (size_t)b * DF_SLOT;
  uint8_t *dst = out + off[b];
  const uint32_t n = len[b];
  if (restart_after(b, nblocks, restart, final_) && threadIdx.x < kRestartMarkerLen) {
    const uint32_t i = threadIdx.x % 5;
    dst[n + threadIdx.x] = i < 3 ? 0 : 0xFF;
  }
  // destination-aligned 4-byte words built from the (aligned) source with a byte shift
  const uint32_t mis = (uint32_t)(reinterpret_cast<uintptr_t>(dst) & 3);
  const uint32_t head = mis ? 4 - mis : 0;
  for (uint32_t i = threadIdx.x; i < head && i < n; i += 256) dst[i] = src[i];
  if (n > head) {
    const uint32_t nw = (n - head) >> 2;
    uint32_t *dw = reinterpret_cast<uint32_t *>(dst + head);
    const uint32_t *sw = reinterpret_cast<const uint32_t *>(src);
    const uint32_t sh = head;  // source byte offset of dst word 0 (0..3)
    for (uint32_t i = threadIdx.x; i < nw; i += 256) {
      uint32_t lo = sw[i], hi = sw[i + 1];
      dw[i] = sh ? __builtin_amdgcn_alignbyte(hi, lo, sh) : lo;
    }
    for (uint32_t i = head + nw * 4 + threadIdx.x; i < n; i += 256) dst[i] = src[i];
  }
}

__global__ void write_bytes(uint8_t *dst, uint64_t v, uint32_t n) {
  if (threadIdx.x < n) dst[threadIdx.x] = (uint8_t)(v >> (8 * threadIdx.x));
}

// reference-style stored blocks (compressionType NONE, src/RawDeflate.ts:93-100,122-153)
__global__ __launch_bounds__(256) void stored_blocks(const uint8_t *__restrict__ in, uint64_t n,
                                                     uint8_t *__restrict__ out, int final_) {
  const uint64_t b = blockIdx.x;
  const uint64_t lo = b * 65535, hi = (lo + 65535) < n ? lo + 65535 : n;
  const uint32_t len = (uint32_t)(hi - lo);
  uint8_t *o = out + b * (65535 + 5);
  if (threadIdx.x == 0) {
    o[0] = (final_ && hi == n) ? 1 : 0;
    o[1] = len & 0xFF;
    o[2] = len >> 8;
    o[3] = (~len) & 0xFF;
    o[4] = ((~len) >> 8) & 0xFF;
  }
  for (uint32_t i = threadIdx.x; i < len; i += 256) o[5 + i] = in[lo + i];
}

}  // namespace

// ---- host launcher ---------------------------------------------------------------------------
struct DeflateLevel {
  int max_chain, nice, lazy, too_far;
};

static DeflateLevel level_params(int level) {
  switch (level) {
    case 1: return {4, 16, 0, 4096};
    case 2: return {8, 32, 0, 4096};
    case 3: return {16, 32, 0, 4096};
    case 4: return {16, 64, 1, 4096};
    case 5: return {32, 128, 1, 4096};
    case 7: return {128, 258, 1, 4096};
    case 8: return {256, 258, 1, 4096};
    case 9: return {1024, 258, 1, 4096};
    default: return {64, 128, 1, 4096};  // 6
  }
}

uint32_t *g_deflate_debug = nullptr;  // test hook (zt_debug_set_deflate_dump)

// Work split: enough workgroups to cover every CU twice, at most 32 blocks
// (1 MiB) per workgroup.  Returns the scratch bytes needed.
static size_t deflate_geometry(const DeviceCtx *c, size_t n, uint32_t *nblocks, uint32_t *k, uint32_t *nwg,
                               size_t *tok_bytes, size_t *slot_bytes, size_t *len_bytes, size_t *off_bytes) {
  *nblocks = (uint32_t)((n + DF_BLOCK - 1) / DF_BLOCK);
  if (*nblocks == 0) *nblocks = 1;
  uint32_t kk = (*nblocks + 2 * c->num_cu - 1) / (2 * c->num_cu);
  uint32_t k2 = 1;
  while (k2 < kk && k2 < 32) k2 <<= 1;  // a power of two, so it divides the restart interval
  kk = k2;
  *k = kk;
  *nwg = (*nblocks + kk - 1) / kk;
  *tok_bytes = (size_t)*nwg * DF_BLOCK * 4;
  *slot_bytes = (size_t)*nblocks * DF_SLOT;
  *len_bytes = ((size_t)*nblocks * 4 + 255) & ~size_t(255);
  *off_bytes = ((size_t)(*nblocks + 1) * 8 + 255) & ~size_t(255);
  return *tok_bytes + *slot_bytes + *len_bytes + *off_bytes + 256;
}

size_t deflate_bound_bytes(size_t n) {
  size_t nb = (n + DF_BLOCK - 1) / DF_BLOCK;
  return n + nb * 16 + (nb / kRestartBlocks + 1) * kRestartMarkerLen + 64;
}

int deflate_dev_run(DeviceCtx *c, const uint8_t *d_in, size_t n, size_t halo, int final_, int ctype, int level,
                    uint8_t *d_out, size_t *out_len, void *scratch_base, size_t scratch_size, hipStream_t s) {
  if (ctype == 0) {
    // stored blocks of <= 65535 bytes (final one flagged)
    size_t nb = (n + 65534) / 65535;
    if (n == 0) {
      write_bytes<<<1, 64, 0, s>>>(d_out, final_ ? 0xFFFF000001ull : 0xFFFF000000ull, 5);
      ZT_HIP(hipGetLastError());
      *out_len = 5;
      return ZT_OK;
    }
    stored_blocks<<<(unsigned)nb, 256, 0, s>>>(d_in, n, d_out, final_);
    ZT_HIP(hipGetLastError());
    *out_len = n + 5 * nb;
    return ZT_OK;
  }
  if (n == 0) {
    write_bytes<<<1, 64, 0, s>>>(d_out, final_ ? 0xFFFF000001ull : 0xFFFF000000ull, 5);
    ZT_HIP(hipGetLastError());
    *out_len = 5;
    return ZT_OK;
  }
  uint32_t nblocks, k, nwg;
  size_t tok_bytes, slot_bytes, len_bytes, off_bytes;
  const size_t need = deflate_geometry(c, n, &nblocks, &k, &nwg, &tok_bytes, &slot_bytes, &len_bytes, &off_bytes);
  if (need > scratch_size) return set_error(ZT_E_NOMEM, "deflate scratch too small");
  uint8_t *sb = static_cast<uint8_t *>(scratch_base);
  DeflateParams P;
  P.base = d_in - halo;
  P.halo = halo;
  P.end = halo + n;
  P.blocks_per_wg = k;
  P.nblocks = nblocks;
  P.restart = kRestartBlocks;
  P.final_ = final_;
  DeflateLevel L = level_params(level);
  P.max_chain = L.max_chain;
  P.nice_len = L.nice;
  P.lazy = L.lazy;
  P.too_far = L.too_far;
  P.ctype = ctype;
  P.dbg = g_deflate_debug;
  P.tokens = reinterpret_cast<uint32_t *>(sb);
  P.slots = sb + tok_bytes;
  P.slot_len = reinterpret_cast<uint32_t *>(sb + tok_bytes + slot_bytes);
  uint64_t *off = reinterpret_cast<uint64_t *>(sb + tok_bytes + slot_bytes + len_bytes);
  ZT_TRY(timing_begin(c, s));
  deflate_kernel<<<nwg, DF_THREADS, 0, s>>>(P);
  ZT_HIP(hipGetLastError());
  ZT_TRY(timing_end(c, s));
  scan_sizes<<<1, 1024, 0, s>>>(P.slot_len, nblocks, off, 0, P.restart, final_);
  ZT_HIP(hipGetLastError());
  gather_blocks<<<nblocks, 256, 0, s>>>(P.slots, P.slot_len, off, d_out, nblocks, P.restart, final_);
  ZT_HIP(hipGetLastError());
  uint64_t total = 0;
  ZT_HIP(hipMemcpyAsync(&total, off + nblocks, sizeof total, hipMemcpyDeviceToHost, s));
  ZT_HIP(hipStreamSynchronize(s));
  ZT_TRY(timing_collect(c, &c->times.deflate_ms, &c->times.deflate_launches));
  *out_len = total;
  return ZT_OK;
}

#ifdef ZT_DF_PROF
extern "C" int zt_debug_deflate_prof(unsigned long long *out) {
  hipMemcpyFromSymbol(out, HIP_SYMBOL(g_df_prof), sizeof(unsigned long long) * 8);
  unsigned long long z[8] = {};
  hipMemcpyToSymbol(HIP_SYMBOL(g_df_prof), z, sizeof z);
  return 0;
}
#endif

size_t deflate_scratch_bytes(const DeviceCtx *c, size_t n) {
  uint32_t nb, k, nwg;
  size_t a, b2, l, o;
  return deflate_geometry(c, n, &nb, &k, &nwg, &a, &b2, &l, &o);
}

}  // namespace zt
