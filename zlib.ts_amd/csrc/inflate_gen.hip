// inflate_gen.hip -- parallel inflate of streams WITHOUT sync points: the
// reference's own RawDeflate output (the whole input as one dynamic block,
// src/RawDeflate.ts:105-107) and zlib / gzip output (many blocks, none byte
// aligned).  Replaces src/RawInflate.ts:127-143 / :466-516 for such streams;
// results are identical to the sequential decode by construction.
//
//   1. find_blocks / check_headers: every bit position is tested for a
//      dynamic block header (BTYPE 2, HLIT / HDIST in range, a complete
//      code-length code -- bit-parallel filters over 32 positions per lane),
//      survivors are decoded in full (complete literal/length and distance
//      codes, end-of-block present); every byte for a stored block's
//      LEN / NLEN pair.  Candidates are hints: a false one costs time, never
//      correctness.
//   2. The stream is cut into cells of C bits.  A cell's unit starts at its
//      first candidate (a guessed block start), else at the cell start
//      *inside* a block: Huffman tables from the nearest preceding candidate
//      header (or a stored payload with the bytes it has left).
//      gen_tokenize_kernel decodes each unit with one wave (the 64-lane SIMT
//      body decoder of inflate_simt.h) until the first token / block start at
//      or after the next unit's start, and records the end state; units that
//      start inside a body record where their path's tokens start.
//   3. gen_link_kernel: unit k continues unit k-1 when k-1's end state is
//      k's start state -- exactly, or for an inside-body start: the same
//      block and a token start of k's path (Huffman codes resynchronise, so
//      the speculative path merges with the true one within a few tokens).
//      The host walks the chain from the stream start; units that do not
//      link are decoded again from their predecessor's end state (exact),
//      and units that guessed a header the chain proved false are guessed
//      again.  A few passes converge; otherwise the one-wave decoder runs.
//   4. expand_kernel (inflate_tok.hip) in marker mode, then
//      copy_marker_kernel per ~1 MiB output segment with a u16 LDS history
//      ring: bytes whose source lies before the segment are written as
//      window markers (0x8000 | position in the previous segment's last
//      32 KiB); window_chain_kernel resolves the 32 KiB windows segment after
//      segment (one workgroup, windows in LDS); marker_resolve_kernel writes
//      the final bytes.
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "inflate_simt.h"

namespace zt {

namespace {

bool gen_debug() {
  static const bool on = getenv("ZT_INF_DEBUG") != nullptr;
  return on;
}
#define GFALLBACK(...)                                                 \
  do {                                                                 \
    if (gen_debug()) fprintf(stderr, "[zt inflate gen] " __VA_ARGS__); \
    return 1;                                                          \
  } while (0)

constexpr uint32_t kMaxCandB = 1u << 24;  // stage-B survivors (Kraft-complete code-length codes)
constexpr uint32_t kMaxCand = 1u << 22;   // validated candidates
constexpr uint32_t GEN_BM_WORDS = SP_WORDS * 64;  // one round of token starts (head or tail)
#ifndef ZT_GEN_OVERLAP
#define ZT_GEN_OVERLAP 8192
#endif
constexpr uint32_t GEN_OVERLAP = ZT_GEN_OVERLAP;   // bits decoded past a GK_HUFF stop for the successor's merge
constexpr uint64_t kNoStop = ~0ull;

// dword `wi` of the 16-byte aligned base, bytes outside [lo, hi) as 0
__device__ __forceinline__ uint32_t ldw(g_u32 *a32, int64_t wi, uint64_t lo, uint64_t hi) {
  if (wi < 0 || (uint64_t)wi * 4 >= hi) return 0u;
  uint32_t v = a32[wi];
  const uint64_t b = (uint64_t)wi * 4;
  if (b < lo || b + 4 > hi) {
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (b + k < lo || b + k >= hi) v &= ~(0xFFu << (8 * k));
  }
  return v;
}

// ---------------------------------------------------------------- 1. candidates
// One lane per dword of input: the 32 bit positions starting in it.  Stage A
// (bit-parallel over the 32 positions): BFINAL any, BTYPE = 2, HLIT <= 29,
// HDIST <= 29.  Stage B per survivor: the HCLEN code-length code lengths form
// a complete prefix code.  Stored blocks: LEN = ~NLEN at a byte whose
// predecessor's top bits are zero padding.
// Each workgroup takes FB_ITER spans of 256 dwords and gathers its stage-B
// survivors in LDS: one atomic on the shared counter per workgroup (one per
// wave serialised at the counter's L2 slice: 1.35 ms of a 64 MiB stream's
// general decode, about one survivor per wave).
constexpr int FB_ITER = 8;
constexpr int FB_LOCAL = 1024;  // survivors a workgroup gathers (more: per-wave atomics)
__global__ __launch_bounds__(256) void find_blocks(const uint8_t *in, uint64_t n, uint64_t index, uint64_t w_first,
                                                   uint64_t nw, uint64_t *listb, uint32_t *cntb, uint64_t *list,
                                                   uint32_t *cnt) {
  __shared__ uint64_t loc[FB_LOCAL];
  __shared__ uint32_t nloc, gbase;
  if (threadIdx.x == 0) nloc = 0;
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const uintptr_t a = reinterpret_cast<uintptr_t>(in);
  g_u32 *a32 = (g_u32 *)(a & ~uintptr_t(15));
  const uint64_t lo = a & 15, hi = lo + n;
  const uint64_t pmin = (lo + index) * 8;
  const uint64_t pmax = hi * 8 >= 17 ? hi * 8 - 17 : 0;  // a header needs >= 17 bits
  for (int it = 0; it < FB_ITER; ++it) {
    // (every lane runs to the end: the appends are wave-aggregated)
    const uint64_t k = ((uint64_t)blockIdx.x * FB_ITER + it) * 256 + threadIdx.x;
    const int64_t wi = (int64_t)(w_first + (k < nw ? k : nw));
    const uint32_t wm = ldw(a32, wi - 1, lo, hi);
    const uint32_t w0 = ldw(a32, wi, lo, hi), w1 = ldw(a32, wi + 1, lo, hi);
    const uint32_t w2 = ldw(a32, wi + 2, lo, hi), w3 = ldw(a32, wi + 3, lo, hi);
    auto S = [&](int sh) -> uint32_t { return __builtin_amdgcn_alignbit(w1, w0, sh); };
    uint32_t M = ~S(1) & S(2);
    M &= ~(S(4) & S(5) & S(6) & S(7));
    M &= ~(S(9) & S(10) & S(11) & S(12));
    const uint64_t base = (uint64_t)wi * 32;
    if (k >= nw) M = 0;
    if (base < pmin) M = (pmin - base >= 32) ? 0u : (M & (0xFFFFFFFFu << (pmin - base)));
    if (base + 32 > pmax) M = (base >= pmax) ? 0u : (M & (0xFFFFFFFFu >> (32 - (pmax - base))));
    uint32_t B = 0;  // survivors of stage B
    while (M) {
      const int j = __builtin_ctz(M);
      M &= M - 1;
      const uint32_t x0 = j ? __builtin_amdgcn_alignbit(w1, w0, j) : w0;
      const uint32_t x1 = j ? __builtin_amdgcn_alignbit(w2, w1, j) : w1;
      const uint32_t x2 = j ? __builtin_amdgcn_alignbit(w3, w2, j) : w2;
      const uint32_t ncl = ((x0 >> 13) & 15) + 4;
      const uint64_t cl = (((uint64_t)x1 << 32 | x0) >> 17) | ((uint64_t)x2 << 47);
      uint32_t kraft = 0;
#pragma unroll
      for (uint32_t i = 0; i < 19; ++i) {
        const uint32_t l = (uint32_t)(cl >> (3 * i)) & 7;
        kraft += (i < ncl && l) ? (128u >> l) : 0u;
      }
      if (kraft == 128) B |= 1u << j;
    }
    // survivors into the workgroup's LDS list (one LDS atomic per wave), or
    // when it is full straight to the global list
    const uint32_t nbk = __popc(B);
    uint32_t pre = nbk;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const uint32_t v = __shfl_up(pre, off, 64);
      if (lane >= off) pre += v;
    }
    const uint32_t wtot = __shfl(pre, 63, 64);
    if (wtot) {
      uint32_t wb = 0;
      if (lane == 63) wb = atomicAdd(&nloc, wtot);
      wb = __shfl(wb, 63, 64);
      const bool local = wb + wtot <= (uint32_t)FB_LOCAL;
      uint32_t gb = 0;
      if (!local && lane == 63) gb = atomicAdd(cntb, wtot);
      gb = __shfl(gb, 63, 64);
      uint32_t q = pre - nbk;
      while (B) {
        const int j = __builtin_ctz(B);
        B &= B - 1;
        if (local)
          loc[wb + q] = base + j;
        else if (gb + q < kMaxCandB)
          listb[gb + q] = base + j;
        ++q;
      }
    }
    // stored LEN fields at bytes 4 wi + j
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint64_t q = (uint64_t)wi * 4 + j;
      if (k >= nw || q < lo + index + 1 || q + 4 > hi) continue;
      const uint32_t x = j ? __builtin_amdgcn_alignbyte(w1, w0, j) : w0;
      const uint32_t prevb = j ? (w0 >> (8 * (j - 1))) & 0xFF : wm >> 24;
      if (((x ^ (x >> 16)) & 0xFFFF) == 0xFFFF && (prevb >> 6) == 0) {
        const uint32_t c = atomicAdd(cnt, 1u);
        if (c < kMaxCand) list[c] = ((q - lo) * 8) << 17 | (uint64_t)(x & 0xFFFF) << 1 | 1;
      }
    }
  }
  __syncthreads();
  const uint32_t nl = nloc < (uint32_t)FB_LOCAL ? nloc : (uint32_t)FB_LOCAL;
  if (threadIdx.x == 0) gbase = nl ? atomicAdd(cntb, nl) : 0u;
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < nl; i += 256)
    if (gbase + i < kMaxCandB) listb[gbase + i] = loc[i];
}

// Stage C: one lane per survivor -- the dynamic header decoded in full with a
// per-lane 128-entry code-length decode table in LDS: the literal/length
// code complete (or one 1-bit code), end-of-block coded, the distance code
// complete, one 1-bit code or empty (the code sets zlib's inflate accepts).
__global__ __launch_bounds__(256) void check_headers(const uint8_t *in, uint64_t n, const uint64_t *listb,
                                                     const uint32_t *cntb, uint64_t *list, uint32_t *cnt) {
  __shared__ uint8_t lut[256][128];
  const uint32_t nb = min(*cntb, kMaxCandB);
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i >= nb) return;
  const uintptr_t a = reinterpret_cast<uintptr_t>(in);
  g_u32 *a32 = (g_u32 *)(a & ~uintptr_t(15));
  const uint64_t lo = a & 15, hi = lo + n;
  uint64_t q = listb[i];
  const uint64_t p0 = q;
  auto bits = [&](uint32_t nbits) -> uint32_t {  // nbits <= 24
    const int64_t wi = (int64_t)(q >> 5);
    const uint64_t v = ((uint64_t)ldw(a32, wi + 1, lo, hi) << 32) | ldw(a32, wi, lo, hi);
    const uint32_t r = (uint32_t)(v >> (q & 31)) & ((1u << nbits) - 1);
    q += nbits;
    return r;
  };
  const uint32_t h = bits(17);
  const uint32_t hlit = ((h >> 3) & 31) + 257, hdist = ((h >> 8) & 31) + 1, ncl = ((h >> 13) & 15) + 4;
  uint8_t *L = lut[threadIdx.x];
  // code-length code: lengths by symbol, canonical codes, reversed into the table
  uint64_t lens = 0;  // 3 bits per symbol
  for (uint32_t k = 0; k < ncl; ++k) lens |= (uint64_t)bits(3) << (3 * kClOrder[k]);
  uint32_t cntl[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int s = 0; s < 19; ++s) cntl[(lens >> (3 * s)) & 7]++;
  uint32_t next[8];
  uint32_t code = 0;
  cntl[0] = 0;
  for (int l = 1; l < 8; ++l) {
    code = (code + cntl[l - 1]) << 1;
    next[l] = code;
  }
  for (int s = 0; s < 19; ++s) {
    const uint32_t l = (uint32_t)(lens >> (3 * s)) & 7;
    if (!l) continue;
    const uint32_t c = next[l]++;
    const uint32_t r = __brev(c) >> (32 - l);
    for (uint32_t f = r; f < 128; f += 1u << l) L[f] = (uint8_t)(s | (l << 5));
  }
  const uint32_t total = hlit + hdist;
  uint32_t k = 0, prev = 0, lsum = 0, dsum = 0, lcodes = 0, dcodes = 0, eob = 0;
  bool ok = true;
  while (k < total) {
    if (q > hi * 8) {
      ok = false;
      break;
    }
    const int64_t wi = (int64_t)(q >> 5);
    const uint64_t v = ((uint64_t)ldw(a32, wi + 1, lo, hi) << 32) | ldw(a32, wi, lo, hi);
    const uint32_t e = L[(uint32_t)(v >> (q & 31)) & 127];
    q += e >> 5;
    const uint32_t sym = e & 31;
    uint32_t rep = 1, len = sym;
    if (sym == 16) {
      if (k == 0) {
        ok = false;
        break;
      }
      rep = 3 + bits(2);
      len = prev;
    } else if (sym == 17) {
      rep = 3 + bits(3);
      len = 0;
    } else if (sym == 18) {
      rep = 11 + bits(7);
      len = 0;
    }
    prev = len;
    if (k + rep > total) {
      ok = false;
      break;
    }
    if (len) {
      const uint32_t nl = k < hlit ? min(hlit - k, rep) : 0u;
      const uint32_t nd = rep - nl;
      lsum += nl << (15 - len);
      dsum += nd << (15 - len);
      lcodes += nl;
      dcodes += nd;
      if (k <= 256 && 256 < k + rep) eob = len;
      if (lsum > 32768 || dsum > 32768) {
        ok = false;
        break;
      }
    }
    k += rep;
  }
  if (!ok || !eob) return;
  if (!(lsum == 32768 || (lcodes == 1 && lsum == 16384))) return;
  if (!(dsum == 32768 || dcodes == 0 || (dcodes == 1 && dsum == 16384))) return;
  const uint32_t c = atomicAdd(cnt, 1u);
  if (c < kMaxCand) list[c] = (p0 - lo * 8) << 17;
}

// ---------------------------------------------------------------- 2. units
struct GenShared {
  uint32_t inbuf[IN_RING_WORDS + 4];
  HuffTab lit;
  HuffTab dist;
  uint8_t lens[320];
};

struct GenParams {
  const uint8_t *in;
  uint64_t n;
  const GenJob *jobs;
  GenResult *res;
  const uint32_t *which;  // units to decode (null: 0 .. count-1)
  uint32_t *tokens;
  uint32_t *bm;           // 2 x GEN_BM_WORDS per unit: head (speculative start), tail (overlap past the stop)
  uint32_t count;
};

__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(3))) void gen_tokenize_kernel(GenParams P) {
  __shared__ GenShared sh;
  __shared__ SpecShared spsh;
  const uint32_t u = P.which ? P.which[blockIdx.x] : blockIdx.x;
  const int lane = threadIdx.x & 63;
  const GenJob job = P.jobs[u];
  GenState st = job.st;
  const uint64_t stop = job.stop;
  Reader rd;
  rd.init(P.in, P.n, min(st.pos >> 3, P.n), sh.inbuf, lane);
  const uint64_t lo8 = rd.lo * 8;
  TokOut to;
  to.tok = P.tokens + job.tok_off;
  to.cap = job.tok_cap;
  to.ntok = 0;
  to.stg = 0;
  to.lane = lane;
  uint64_t op = 0, dec_start = 0;
  uint32_t recorded = 0, blk_final = 0, tab_final = 0, tail_ok = 0, ntok_stop = 0;
  uint64_t tab_id = 0, out_stop = 0;
  bool stopped_here = false;
  int status = ZT_OK, detail = 0;
  uint64_t tab_hdr = ~0ull;
  g_u8 *gin = (g_u8 *)P.in;
  for (;;) {
    if (st.kind == GK_FINAL) break;
    if (st.kind == GK_BLOCK) {
      if (st.pos >= stop) break;
      rd.seek_bit(lo8 + st.pos);
      uint32_t v;
      if (!rd.template bits<false>(3, v)) {
        status = ZT_E_INPUT_BROKEN;
        break;
      }
      blk_final = v & 1;
      const uint32_t btype = v >> 1;
      if (btype == 0) {
        st.kind = GK_SHDR;
        st.pos = ((rd.pos_bits_in() + 7) >> 3) << 3;
        st.bfinal = blk_final;
        continue;
      }
      status = read_tables<false>(rd, sh.lens, &sh.lit, &sh.dist, btype, lane, detail);
      if (status) break;
      st.hdr = btype == 1 ? kFixedHdr : st.pos;
      tab_hdr = st.hdr;
      st.kind = GK_HUFF;
      st.bfinal = blk_final;
      st.pos = rd.pos_bits_in();
    } else if (st.kind == GK_HUFF && tab_hdr != st.hdr) {
      // start inside a body: the block's tables from its header (fixed
      // codes: the fixed tables, BFINAL from the state)
      if (st.hdr == kFixedHdr) {
        blk_final = st.bfinal;
        status = read_tables<false>(rd, sh.lens, &sh.lit, &sh.dist, 1, lane, detail);
        if (status) break;
        tab_hdr = kFixedHdr;
        rd.seek_bit(lo8 + st.pos);
      } else {
        rd.seek_bit(lo8 + st.hdr);
        uint32_t v;
        if (!rd.template bits<false>(3, v)) {
          status = ZT_E_INPUT_BROKEN;
          break;
        }
        blk_final = v & 1;
        const uint32_t btype = v >> 1;
        if (btype == 0 || btype == 3) {
          status = ZT_E_UNKNOWN_BTYPE;
          detail = (int)btype;
          break;
        }
        status = read_tables<false>(rd, sh.lens, &sh.lit, &sh.dist, btype, lane, detail);
        if (status) break;
        if (btype == 1) st.hdr = kFixedHdr;
        tab_hdr = st.hdr;
        st.bfinal = blk_final;
        const uint64_t body = rd.pos_bits_in();
        if (st.pos < body) st.pos = body;  // a start inside the header: the body's first token
      }
    }
    if (st.kind == GK_HUFF) {
      const bool rec = job.spec && !recorded;
      const uint64_t b = st.pos;
      const uint32_t stop_rel =
          stop == kNoStop ? 0xFFFFFFFFu : (stop <= b ? 0u : (uint32_t)min(stop - b, (uint64_t)0xFFFFFFF0u));
      bool stopped = false;
      uint64_t end_bit = 0;
      const int r = tok_huffman_simt(rd, lo8 + b, &sh.lit, &sh.dist, to, op, &spsh, end_bit, nullptr, stop_rel,
                                     rec ? P.bm + (uint64_t)u * 2 * GEN_BM_WORDS : nullptr, &stopped);
      if (r != 0) {
        status = r == 1 ? ZT_E_INPUT_BROKEN : r;
        break;
      }
      if (rec) {
        dec_start = b;
        recorded = 1;
        tab_id = st.hdr;
        tab_final = blk_final;
      }
      st.pos = end_bit - lo8;
      if (stopped) {
        // the end state; then an overlap past it, whose token starts let a
        // successor that started inside this body find where the paths merge
        ntok_stop = uni(to.ntok);
        out_stop = op;
        bool s2 = false;
        uint64_t e2 = 0;
        const int r2 = tok_huffman_simt(rd, end_bit, &sh.lit, &sh.dist, to, op, &spsh, e2, nullptr, GEN_OVERLAP,
                                        P.bm + (uint64_t)u * 2 * GEN_BM_WORDS + GEN_BM_WORDS, &s2);
        tail_ok = r2 == 0 ? 1u : 0u;
        stopped_here = true;
        break;
      }
      st.kind = blk_final ? GK_FINAL : GK_BLOCK;
      continue;
    }
    if (st.kind == GK_SHDR) {
      if (st.pos >= stop) break;
      const uint64_t q = st.pos >> 3;
      if (q + 4 > P.n) {
        status = ZT_E_STORED_LEN;
        break;
      }
      const uint32_t len = (uint32_t)gin[q] | ((uint32_t)gin[q + 1] << 8);
      const uint32_t nlen = (uint32_t)gin[q + 2] | ((uint32_t)gin[q + 3] << 8);
      if (len != (~nlen & 0xFFFFu)) {
        status = ZT_E_STORED_NLEN;
        break;
      }
      st.kind = GK_STORED;
      st.rem = len;
      st.pos = (q + 4) * 8;
      continue;
    }
    if (st.kind == GK_STORED) {
      if (st.rem == 0) {
        st.kind = st.bfinal ? GK_FINAL : GK_BLOCK;
        continue;
      }
      if (st.pos >= stop) break;
      uint64_t kb = st.rem;
      if (stop != kNoStop && stop < st.pos + 8 * kb) kb = (stop - st.pos + 7) >> 3;
      const uint64_t p = st.pos >> 3;
      if (p + kb > P.n) {
        status = ZT_E_INPUT_BROKEN;
        break;
      }
      const uint32_t len = (uint32_t)kb;
      const uint32_t nt0 = uni(to.ntok);
      if ((uint64_t)nt0 + len > to.cap) {
        status = ZT_E_NOMEM;
        break;
      }
      to.flush_partial();
      for (uint32_t j = lane; j < len; j += 64) to.tok[nt0 + j] = gin[p + j];
      const uint32_t nt = nt0 + len;
      const uint32_t idx = (nt & ~63u) + (uint32_t)lane;
      if ((uint32_t)lane < (nt & 63) && idx >= nt0) to.stg = gin[p + idx - nt0];
      to.ntok = nt;
      op += len;
      st.pos += 8 * kb;
      st.rem -= len;
      continue;
    }
    status = ZT_E_INPUT_BROKEN;  // unknown state kind
    break;
  }
  to.flush_partial();
  if (!stopped_here) {
    ntok_stop = to.ntok;
    out_stop = op;
  }
  if (lane == 0) {
    GenResult r;
    r.end = st;
    r.out_len = op;
    r.out_stop = out_stop;
    r.ntok_stop = ntok_stop;
    r.tail_ok = tail_ok;
    r.dec_start = dec_start;
    r.ntok = to.ntok;
    r.status = status;
    r.detail = detail;
    r.recorded = recorded;
    r.tab_id = tab_id;
    r.tab_final = tab_final;
    r.pad = 0;
    P.res[u] = r;
  }
}

__device__ __forceinline__ bool same_state(const GenState &a, const GenState &b) {
  if (a.kind != b.kind || a.pos != b.pos) return false;
  if (a.kind == GK_HUFF) return a.hdr == b.hdr && a.bfinal == b.bfinal;
  if (a.kind == GK_STORED) return a.rem == b.rem && a.bfinal == b.bfinal;
  if (a.kind == GK_SHDR) return a.bfinal == b.bfinal;
  return true;
}

// ---------------------------------------------------------------- 3. links
// bits [off, off + 32) of a bitmap of GEN_BM_WORDS words (0 outside)
__device__ __forceinline__ uint32_t bm_bits(const uint32_t *b, int64_t off) {
  if (off <= -32 || off >= (int64_t)GEN_BM_WORDS * 32) return 0u;
  const int64_t w = off >> 5;  // floor
  const uint32_t sh = (uint32_t)(off & 31);
  const uint32_t lo = (w >= 0) ? b[w] : 0u;
  const uint32_t hi = (w + 1 < (int64_t)GEN_BM_WORDS && w + 1 >= 0) ? b[w + 1] : 0u;
  return sh ? __builtin_amdgcn_alignbit(hi, lo, sh) : lo;
}

// sum of the output lengths of tokens [a, b)
__device__ __forceinline__ uint64_t tok_bytes(const uint32_t *tk, uint32_t a, uint32_t b, int lane) {
  uint64_t s = 0;
  for (uint32_t i = a + lane; i < b; i += 64) {
    const uint32_t v = tk[i];
    s += (v >> 16) ? (v >> 16) : 1u;
  }
  for (int off = 32; off; off >>= 1) s += __shfl_xor(s, off, 64);
  return s;
}

// unit k against unit k-1: an exact start state joins at k-1's end state; a
// start inside a body joins at the first token start both paths share --
// k-1's overlap past its end (tail) and k's speculative path (head)
__global__ __launch_bounds__(64) void gen_link_kernel(const GenJob *jobs, const GenResult *res, const uint32_t *bm,
                                                      const uint32_t *tokens, const uint32_t *which, GenLink *link) {
  const uint32_t k = which[blockIdx.x];
  const int lane = threadIdx.x & 63;
  const GenResult pr = res[k - 1];
  const GenState prev = pr.end;
  const GenJob job = jobs[k];
  const GenResult r = res[k];
  uint32_t ok = 0, t = 0, cut = pr.ntok_stop;
  uint64_t bytes = 0, pbytes = pr.out_stop;
  if (job.st.kind == GK_HUFF && job.spec) {
    if (prev.kind == GK_HUFF && prev.hdr == r.tab_id && prev.bfinal == r.tab_final && r.recorded && pr.tail_ok) {
      const uint32_t *tail = bm + (uint64_t)(k - 1) * 2 * GEN_BM_WORDS + GEN_BM_WORDS;
      const uint32_t *head = bm + (uint64_t)k * 2 * GEN_BM_WORDS;
      const int64_t d = (int64_t)prev.pos - (int64_t)r.dec_start;  // head offset of tail bit 0
      uint32_t best = 0xFFFFFFFFu;  // first tail bit set in both
      for (uint32_t w = lane; w < GEN_BM_WORDS; w += 64) {
        const uint32_t m = tail[w] & bm_bits(head, d + 32 * (int64_t)w);
        if (m) {
          best = 32 * w + __builtin_ctz(m);
          break;
        }
      }
      for (int off = 32; off; off >>= 1) best = min(best, (uint32_t)__shfl_xor((int)best, off, 64));
      if (best != 0xFFFFFFFFu) {
        // tokens before the join: k-1's overlap marks below `best`, k's head marks below d + best
        uint32_t c1 = 0, c2 = 0;
        for (uint32_t w = lane; w * 32 < best; w += 64) {
          uint32_t m = tail[w];
          if (w * 32 + 32 > best) m &= (1u << (best & 31)) - 1;
          c1 += __popc(m);
        }
        const int64_t hb = d + (int64_t)best;  // head bit of the join (>= 0)
        for (int64_t w = lane; w * 32 < hb; w += 64) {
          uint32_t m = head[w];
          if (w * 32 + 32 > hb) m &= (1u << (hb & 31)) - 1;
          c2 += __popc(m);
        }
        for (int off = 32; off; off >>= 1) {
          c1 += __shfl_xor(c1, off, 64);
          c2 += __shfl_xor(c2, off, 64);
        }
        cut = pr.ntok_stop + c1;
        t = c2;
        if (hb >= 0 && cut <= pr.ntok && t <= r.ntok) {
          ok = 1;
          pbytes = pr.out_stop + tok_bytes(tokens + jobs[k - 1].tok_off, pr.ntok_stop, cut, lane);
          bytes = tok_bytes(tokens + job.tok_off, 0, t, lane);
        }
      }
    }
  } else {
    ok = same_state(prev, job.st) ? 1u : 0u;
  }
  if (lane == 0) {
    GenLink l;
    l.bytes = bytes;
    l.prev_bytes = pbytes;
    l.ok = ok;
    l.t = t;
    l.prev_cut = cut;
    l.pad = 0;
    link[k] = l;
  }
}

// ---------------------------------------------------------------- 4. bytes
// copy_kernel (inflate_tok.hip) with a u16 history ring: a ring entry is a
// byte (< 0x100) or a window marker 0x8000 | w, "byte w of the 32 KiB before
// this segment".  The ring starts as the markers of that window.
typedef unsigned int u32x4g __attribute__((ext_vector_type(4)));

struct CopyShared16 {
  uint16_t ring[RING];
  uint16_t desc[CP_DESC_RING];
};

__device__ __forceinline__ uint32_t cp_val16(const CopyShared16 *sh, uint64_t op, uint32_t d, int32_t &off) {
  const uint32_t rv = sh->ring[((uint32_t)op - d - 1) & RING_MASK];
  const bool lit = (d & 0x8000u) != 0;
  off = (lit && (d & 0x4000u)) ? (int32_t)(d & 0x3FF) : -1;
  return lit ? (d & 0xFF) : rv;
}

__device__ __forceinline__ void cp_flush16(const CopyShared16 *sh, uint16_t *out, uint64_t lo, uint64_t hi, int lane) {
  if (lo >= hi) return;
  const uint64_t hv = lo + ((hi - lo) & ~uint64_t(7));
  for (uint64_t p = lo + (uint64_t)lane * 8; p < hv; p += 512)
    *reinterpret_cast<u32x4g *>(out + p) = *reinterpret_cast<const u32x4g *>(&sh->ring[p & RING_MASK]);
  for (uint64_t p = hv + lane; p < hi; p += 64) out[p] = sh->ring[p & RING_MASK];
}

__global__ __launch_bounds__(64) void copy_marker_kernel(ResolveParams P, const GenSeg *gs, uint16_t *out16) {
  __shared__ CopyShared16 sh;
  const uint32_t sg = blockIdx.x;
  const int lane = threadIdx.x & 63;
  const SegJob sj = P.segs[sg];
  const GenSeg g = gs[sg];
  const uint64_t n = g.len;
  uint16_t *out = out16 + g.base16;
  const uint16_t *dsrc = P.desc + P.units[sj.first].desc_off;
  for (uint32_t i = (uint32_t)lane * 4; i < (uint32_t)RING; i += 256) {
    const uint64_t m = sg ? ((uint64_t)(0x8000u | i) | ((uint64_t)(0x8001u | i) << 16) |
                             ((uint64_t)(0x8002u | i) << 32) | ((uint64_t)(0x8003u | i) << 48))
                          : 0ull;
    *reinterpret_cast<uint64_t *>(&sh.ring[i]) = m;
  }
  wave_sync();
  uint64_t issued = 0, flushed = 0;
  for (uint64_t op = 0; op < n; op += CP_STEP) {
    cp_desc_fetch(dsrc, sh.desc, op, n, issued, lane);
    uint64_t dd[CP_G];
#pragma unroll
    for (int g = 0; g < CP_G; ++g) {
      const uint32_t x = (uint32_t)op + 256u * g + 4 * (uint32_t)lane;
      dd[g] = *reinterpret_cast<const uint64_t *>(&sh.desc[x & (CP_DESC_RING - 1)]);
    }
    uint64_t bw[CP_G];
    bool in_step = false;
#pragma unroll
    for (int g = 0; g < CP_G; ++g) {
      int32_t o0, o1, o2, o3;
      const uint32_t b0 = cp_val16(&sh, op, (uint32_t)dd[g] & 0xFFFF, o0);
      const uint32_t b1 = cp_val16(&sh, op, (uint32_t)(dd[g] >> 16) & 0xFFFF, o1);
      const uint32_t b2 = cp_val16(&sh, op, (uint32_t)(dd[g] >> 32) & 0xFFFF, o2);
      const uint32_t b3 = cp_val16(&sh, op, (uint32_t)(dd[g] >> 48), o3);
      bw[g] = (uint64_t)b0 | ((uint64_t)b1 << 16) | ((uint64_t)b2 << 32) | ((uint64_t)b3 << 48);
      in_step = in_step || o0 >= 0 || o1 >= 0 || o2 >= 0 || o3 >= 0;
    }
    if (__ballot(in_step) == 0) {
#pragma unroll
      for (int g = 0; g < CP_G; ++g)
        *reinterpret_cast<uint64_t *>(&sh.ring[((uint32_t)op + 256u * g + 4 * (uint32_t)lane) & RING_MASK]) = bw[g];
    } else {
      for (uint32_t sub = 0; sub < CP_STEP; sub += 64) {
        const uint64_t y = op + sub + (uint64_t)lane;
        const uint32_t d = y < n ? sh.desc[y & (CP_DESC_RING - 1)] : 0x8000u;
        int32_t off;
        uint32_t val = cp_val16(&sh, op, d, off);
        int32_t ptr = -1;
        if (off >= (int32_t)(sub + lane)) off = -1;
        if (off >= 0) {
          if ((uint32_t)off < sub)
            val = sh.ring[(op + off) & RING_MASK];
          else
            ptr = off - (int32_t)sub;
        }
        while (__ballot(ptr >= 0)) {
          const uint32_t q = ptr >= 0 ? (uint32_t)ptr : (uint32_t)lane;
          const uint32_t v2 = bperm(val, q);
          const int32_t p2 = (int32_t)bperm((uint32_t)ptr, q);
          if (ptr >= 0) {
            if (p2 < 0) {
              val = v2;
              ptr = -1;
            } else {
              ptr = p2;
            }
          }
        }
        sh.ring[y & RING_MASK] = (uint16_t)val;
        wave_sync();
      }
    }
    wave_sync();
    const uint64_t end = op + CP_STEP < n ? op + CP_STEP : n;
    if (end - flushed >= RS_FLUSH) {
      const uint64_t upto = flushed + RS_FLUSH;
      cp_flush16(&sh, out, flushed, upto, lane);
      flushed = upto;
    }
  }
  wave_sync();
  cp_flush16(&sh, out, flushed, n, lane);
  if (lane == 0) P.seg_status[sg] = ZT_OK;
}

// The 32 KiB window after each segment, in order: window j = the last 32 KiB
// of segment j with its markers looked up in window j - 1 (kept in LDS).
// Thread t owns entries [32 t, 32 t + 32); the next segment's tail is loaded
// while this one resolves, so a step costs its LDS lookups and one barrier.
__device__ __forceinline__ void wc_load(const GenSeg *gs, uint32_t j, uint32_t nwin, const uint16_t *out16,
                                        uint32_t tid, u32x4g *v) {
  if (j >= nwin) return;
  const GenSeg g = gs[j];
  if (g.len < (uint64_t)RING) return;  // short segment: resolved entry by entry
  const u32x4g *p = reinterpret_cast<const u32x4g *>(out16 + g.base16 + (g.len - RING) + 32 * tid);
  const uintptr_t al = reinterpret_cast<uintptr_t>(p) & 15;
  if (al == 0) {
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] = p[k];
  } else {
    const uint16_t *e = out16 + g.base16 + (g.len - RING) + 32 * tid;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      v[k].x = e[8 * k] | ((uint32_t)e[8 * k + 1] << 16);
      v[k].y = e[8 * k + 2] | ((uint32_t)e[8 * k + 3] << 16);
      v[k].z = e[8 * k + 4] | ((uint32_t)e[8 * k + 5] << 16);
      v[k].w = e[8 * k + 6] | ((uint32_t)e[8 * k + 7] << 16);
    }
  }
}

__global__ __launch_bounds__(1024) void window_chain_kernel(const GenSeg *gs, uint32_t nwin, const uint16_t *out16,
                                                            uint8_t *wins) {
  __shared__ uint32_t w[2][RING / 4];
  const uint32_t tid = threadIdx.x;
  u32x4g cur[4], nxt[4];
  wc_load(gs, 0, nwin, out16, tid, cur);
  for (uint32_t j = 0; j < nwin; ++j) {
    uint32_t *cw = w[j & 1];
    const uint8_t *prv = reinterpret_cast<const uint8_t *>(w[(j & 1) ^ 1]);
    wc_load(gs, j + 1, nwin, out16, tid, nxt);
    const GenSeg g = gs[j];
    uint32_t o[8];
    if (g.len >= (uint64_t)RING) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const uint32_t e[4] = {cur[k].x, cur[k].y, cur[k].z, cur[k].w};
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          uint32_t r = 0;
#pragma unroll
          for (int b = 0; b < 4; ++b) {
            const uint32_t x = (e[2 * h + (b >> 1)] >> (16 * (b & 1))) & 0xFFFF;
            const uint32_t v = (x & 0x8000u) ? prv[x & 0x7FFF] : x;
            r |= (v & 0xFF) << (8 * b);
          }
          o[2 * k + h] = r;
        }
      }
    } else {
      const uint16_t *src = out16 + g.base16;
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        uint32_t r = 0;
        for (int b = 0; b < 4; ++b) {
          const uint32_t i = 32 * tid + 4 * q + b;
          const int64_t p = (int64_t)g.len - RING + i;
          uint32_t v;
          if (p >= 0) {
            const uint32_t x = src[p];
            v = (x & 0x8000u) ? prv[x & 0x7FFF] : x;
          } else {
            v = j ? prv[i + g.len] : 0u;
          }
          r |= (v & 0xFF) << (8 * b);
        }
        o[q] = r;
      }
    }
#pragma unroll
    for (int q = 0; q < 8; ++q) cw[8 * tid + q] = o[q];
    u32x4g *gw = reinterpret_cast<u32x4g *>(wins + (uint64_t)j * RING + 32 * tid);
    gw[0] = u32x4g{o[0], o[1], o[2], o[3]};
    gw[1] = u32x4g{o[4], o[5], o[6], o[7]};
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 4; ++k) cur[k] = nxt[k];
  }
}

// The windows by pointer jumping instead (wj_*): every window entry is a
// byte or a reference (window k, offset w) -- a marker of segment j refers to
// window j - 1, and the head of a window shorter than 32 KiB is the previous
// window's tail -- and each round replaces every reference by what it points
// to, so a chain of k windows resolves in ceil(log2 k) + 1 rounds, each a
// parallel pass over all windows (the serial chain above took ~3.7 us per
// window: 1.9 ms for 512).  Entry: bit 31 = a byte (bits 0-7), else
// (k << 15) | w with k < 2^16.
constexpr uint32_t WJ_BYTE = 0x80000000u;
constexpr uint32_t WJ_MAXWIN = 1u << 16;

__global__ __launch_bounds__(256) void wj_init_kernel(const GenSeg *__restrict__ gs, uint32_t nwin,
                                                      const uint16_t *__restrict__ out16, uint32_t *__restrict__ e) {
  const uint64_t t = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  const uint64_t x0 = t * 4;
  if (x0 >= (uint64_t)nwin * RING) return;
  const uint32_t j = (uint32_t)(x0 / RING);
  const GenSeg g = gs[j];
  uint32_t v[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const uint32_t i = (uint32_t)(x0 % RING) + q;
    const int64_t p = (int64_t)g.len - RING + i;
    if (p >= 0) {
      const uint32_t x = out16[g.base16 + p];
      v[q] = (x & 0x8000u) ? (((j - 1) << 15) | (x & 0x7FFFu)) : (WJ_BYTE | (x & 0xFFu));
    } else {
      v[q] = j ? (((j - 1) << 15) | (uint32_t)(i + g.len)) : WJ_BYTE;
    }
  }
  *reinterpret_cast<u32x4g *>(e + x0) = u32x4g{v[0], v[1], v[2], v[3]};
}

// one round: e_out = e_in with each reference replaced by its target; the
// last round writes the window bytes (a reference left there: status error)
__global__ __launch_bounds__(256) void wj_round_kernel(const uint32_t *__restrict__ ein, uint32_t *__restrict__ eout,
                                                       uint32_t nwin, int last, uint8_t *__restrict__ wins,
                                                       int32_t *__restrict__ st) {
  const uint64_t t = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  const uint64_t x0 = t * 4;
  if (x0 >= (uint64_t)nwin * RING) return;
  const u32x4g a = *reinterpret_cast<const u32x4g *>(ein + x0);
  uint32_t v[4] = {a.x, a.y, a.z, a.w};
#pragma unroll
  for (int q = 0; q < 4; ++q)
    if (!(v[q] & WJ_BYTE)) v[q] = ein[(uint64_t)(v[q] >> 15) * RING + (v[q] & 0x7FFFu)];
  if (!last) {
    *reinterpret_cast<u32x4g *>(eout + x0) = u32x4g{v[0], v[1], v[2], v[3]};
    return;
  }
  uint32_t b = 0;
  bool bad = false;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    bad = bad || !(v[q] & WJ_BYTE);
    b |= (v[q] & 0xFFu) << (8 * q);
  }
  *reinterpret_cast<uint32_t *>(wins + x0) = b;
  if (bad) st[0] = ZT_E_INTERNAL;
}

__global__ __launch_bounds__(256) void marker_resolve_kernel(const GenSeg *gs, const uint16_t *out16,
                                                             const uint8_t *wins, uint8_t *out) {
  const uint32_t j = blockIdx.y;
  const GenSeg g = gs[j];
  const uint64_t i0 = ((uint64_t)blockIdx.x * 256 + threadIdx.x) * 16;
  if (i0 >= g.len) return;
  const uint8_t *win = wins + (j ? (uint64_t)(j - 1) * RING : 0);
  const u32x4g *s = reinterpret_cast<const u32x4g *>(out16 + g.base16 + i0);
  const u32x4g v0 = s[0], v1 = s[1];
  uint32_t x[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
  uint8_t *o = out + g.out_off + i0;
  const uint32_t cnt = g.len - i0 < 16 ? (uint32_t)(g.len - i0) : 16u;
  uint8_t b[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const uint32_t e = (x[k >> 1] >> (16 * (k & 1))) & 0xFFFF;
    b[k] = (uint8_t)((e & 0x8000u) ? win[e & 0x7FFF] : e);
  }
  if (cnt == 16 && ((reinterpret_cast<uintptr_t>(o) & 15) == 0)) {
    u32x4g r;
    r.x = b[0] | (b[1] << 8) | (b[2] << 16) | ((uint32_t)b[3] << 24);
    r.y = b[4] | (b[5] << 8) | (b[6] << 16) | ((uint32_t)b[7] << 24);
    r.z = b[8] | (b[9] << 8) | (b[10] << 16) | ((uint32_t)b[11] << 24);
    r.w = b[12] | (b[13] << 8) | (b[14] << 16) | ((uint32_t)b[15] << 24);
    *reinterpret_cast<u32x4g *>(o) = r;
  } else {
    for (uint32_t k = 0; k < cnt; ++k) o[k] = b[k];
  }
}

size_t al256(size_t v) { return (v + 255) & ~size_t(255); }

void radix_sort64(std::vector<uint64_t> &v, uint64_t max_key) {
  std::vector<uint64_t> tmp(v.size());
  for (int sh = 0; sh < 64 && (max_key >> sh); sh += 11) {
    std::vector<uint32_t> cnt(2049, 0);
    for (uint64_t e : v) ++cnt[((e >> sh) & 2047) + 1];
    for (int i = 0; i < 2048; ++i) cnt[i + 1] += cnt[i];
    for (uint64_t e : v) tmp[cnt[(e >> sh) & 2047]++] = e;
    v.swap(tmp);
  }
}

}  // namespace

// Host orchestration (see the file header).  Returns 0 with the output in
// *d_out_io, 1 when the caller should decode with one wave (errors on the
// chain -- the one-wave decoder reports them exactly -- or no convergence),
// or a negative status.
int inflate_general_dev(DeviceCtx *c, const uint8_t *d_in, size_t n, size_t index, uint8_t **d_out_io,
                        size_t out_cap, size_t *out_len, size_t *end_ip, hipStream_t s) {
  if (n < index + (1u << 14)) return 1;
  const uint64_t bit0 = (uint64_t)index * 8, bitn = (uint64_t)n * 8;
  // ---- 1. candidates
  const uintptr_t ia = reinterpret_cast<uintptr_t>(d_in);
  const uint64_t lo = ia & 15;
  const uint64_t w_first = (lo + index) / 4, w_end = (lo + n + 3) / 4;
  const uint64_t nw = w_end - w_first;
  void *d_c;
  const size_t listb_bytes = (size_t)kMaxCandB * 8, list_bytes = (size_t)kMaxCand * 8;
  ZT_TRY(scratch(c, 10, 256 + listb_bytes + list_bytes, &d_c));
  uint32_t *d_cnt = static_cast<uint32_t *>(d_c);  // [0] stage B, [1] final
  uint64_t *d_listb = reinterpret_cast<uint64_t *>(static_cast<uint8_t *>(d_c) + 256);
  uint64_t *d_list = reinterpret_cast<uint64_t *>(static_cast<uint8_t *>(d_c) + 256 + listb_bytes);
  ZT_TRY(timing_begin(c, s, 2));
  ZT_HIP(hipMemsetAsync(d_cnt, 0, 8, s));
  find_blocks<<<(uint32_t)((nw + 256 * FB_ITER - 1) / (256 * FB_ITER)), 256, 0, s>>>(d_in, n, index, w_first, nw,
                                                                                    d_listb, d_cnt, d_list,
                                                           d_cnt + 1);
  ZT_HIP(hipGetLastError());
  uint32_t cnts[2];
  ZT_TRY(readback(c, cnts, d_cnt, 8, s));
  const uint32_t nb = std::min(cnts[0], kMaxCandB);
  if (nb) {
    check_headers<<<(nb + 255) / 256, 256, 0, s>>>(d_in, n, d_listb, d_cnt, d_list, d_cnt + 1);
    ZT_HIP(hipGetLastError());
  }
  ZT_TRY(readback(c, cnts, d_cnt, 8, s));
  const uint32_t nc = std::min(cnts[1], kMaxCand);
  std::vector<uint64_t> cand(nc);
  if (nc) ZT_TRY(readback(c, cand.data(), d_list, (size_t)nc * 8, s));
  radix_sort64(cand, (bitn << 17) | 0x1FFFF);  // entry: bit position << 17 | stored LEN << 1 | stored
  // stored candidates are hints with false positives (LEN = ~NLEN inside any
  // data): keep one only when a candidate starts where its payload ends (the
  // next block), or the payload ends at the stream end
  {
    std::vector<uint64_t> keep;
    keep.reserve(cand.size());
    auto has = [&](uint64_t pos, bool stored) {
      auto it = std::lower_bound(cand.begin(), cand.end(), pos << 17);
      for (; it != cand.end() && (*it >> 17) == pos; ++it)
        if ((bool)(*it & 1) == stored) return true;
      return false;
    };
    for (uint64_t e : cand) {
      if (!(e & 1)) {
        keep.push_back(e);
        continue;
      }
      const uint64_t q = (e >> 17) >> 3, nxt = q + 4 + ((e >> 1) & 0xFFFF);
      if (nxt + 8 >= (uint64_t)n || has(nxt * 8, false) || has((nxt + 1) * 8, true)) keep.push_back(e);
    }
    cand.swap(keep);
  }
  // ---- 2. units on a grid of cells
  // cells: about 4 units per tokenize slot (8 per CU), 32 K .. 256 K bits
  uint64_t cell = ((bitn - bit0) / (32 * (uint64_t)std::max(c->num_cu, 1))) & ~uint64_t(7);
  if (getenv("ZT_GEN_CELL")) cell = (uint64_t)atoll(getenv("ZT_GEN_CELL")) * 8;
  cell = std::min<uint64_t>(std::max<uint64_t>(cell, 1u << 15), 1u << 18);
  const uint64_t min_gap = 1u << 14;  // a unit spans at least this many bits (room for its successor to merge)
  std::vector<GenJob> jobs;
  std::vector<uint64_t> srcs;  // the candidate each guess came from (~0: exact start)
  {
    GenJob j0{};
    j0.st.kind = GK_BLOCK;
    j0.st.pos = bit0;
    j0.spec = 0;
    jobs.push_back(j0);
    srcs.push_back(~0ull);
  }
  size_t ci = 0;
  int64_t last_dyn = -1, last_st = -1;  // latest candidates below the unit start (indices into cand)
  for (uint64_t x0 = bit0 + cell; x0 < bitn; x0 += cell) {
    const uint64_t lo_pos = jobs.back().st.pos + min_gap;
    if (x0 + cell <= lo_pos) continue;
    const uint64_t x = std::max(x0, (lo_pos + 7) & ~uint64_t(7));
    if (x >= bitn) break;
    while (ci < cand.size() && (cand[ci] >> 17) < x) {
      if (cand[ci] & 1)
        last_st = (int64_t)ci;
      else
        last_dyn = (int64_t)ci;
      ++ci;
    }
    GenJob j{};
    j.spec = 1;
    uint64_t src;
    if (ci < cand.size() && (cand[ci] >> 17) < x0 + cell && (cand[ci] >> 17) < bitn) {
      const uint64_t p = cand[ci] >> 17;
      j.st.kind = (cand[ci] & 1) ? GK_SHDR : GK_BLOCK;
      j.st.pos = p;
      j.st.bfinal = 0;
      src = p;
    } else {
      // inside a block: a stored payload that covers x, else Huffman tables
      // from the nearest dynamic header below (the stream start if none)
      bool done = false;
      if (last_st >= 0 && (last_dyn < 0 || cand[last_st] > cand[last_dyn])) {
        const uint64_t q = (cand[last_st] >> 17) >> 3;
        const uint64_t pend = (q + 4 + ((cand[last_st] >> 1) & 0xFFFF)) * 8;
        if (x < pend) {
          j.st.kind = GK_STORED;
          j.st.pos = x;
          j.st.rem = (uint32_t)((pend - x) >> 3);
          j.st.bfinal = 0;
          done = true;
        }
      }
      if (done) {
        src = cand[last_st] >> 17;
      } else {
        j.st.kind = GK_HUFF;
        j.st.pos = x;
        j.st.hdr = last_dyn >= 0 ? (cand[last_dyn] >> 17) : bit0;
        src = j.st.hdr;
      }
    }
    jobs.push_back(j);
    srcs.push_back(src);
  }
  const size_t units = jobs.size();
  uint64_t tok_total = 0;
  for (size_t k = 0; k < units; ++k) {
    const uint64_t a = jobs[k].st.pos;
    const uint64_t b = k + 1 < units ? jobs[k + 1].st.pos : bitn;
    jobs[k].stop = k + 1 < units ? b : kNoStop;
    uint64_t cap = (b - std::min(a, b)) / 2 + 8192;
    cap = std::min<uint64_t>(cap, 1u << 30);
    jobs[k].tok_off = tok_total;
    jobs[k].tok_cap = (uint32_t)cap;
    tok_total += (cap + 63) & ~uint64_t(63);
  }
  void *d_tok, *d_meta, *d_bm;
  ZT_TRY(scratch(c, 11, (tok_total + 256) * 4, &d_tok));
  const size_t jobs_b = al256(units * sizeof(GenJob)), res_b = al256(units * sizeof(GenResult));
  const size_t link_b = al256(units * sizeof(GenLink)), which_b = al256(units * 4);
  ZT_TRY(scratch(c, 12, jobs_b + res_b + link_b + 2 * which_b, &d_meta));
  ZT_TRY(scratch(c, 13, units * 2 * GEN_BM_WORDS * 4, &d_bm));
  GenJob *d_jobs = static_cast<GenJob *>(d_meta);
  GenResult *d_res = reinterpret_cast<GenResult *>(static_cast<uint8_t *>(d_meta) + jobs_b);
  GenLink *d_link = reinterpret_cast<GenLink *>(static_cast<uint8_t *>(d_meta) + jobs_b + res_b);
  uint32_t *d_which = reinterpret_cast<uint32_t *>(static_cast<uint8_t *>(d_meta) + jobs_b + res_b + link_b);
  uint32_t *d_lwhich = d_which + which_b / 4;
  GenParams gp;
  gp.in = d_in;
  gp.n = n;
  gp.jobs = d_jobs;
  gp.res = d_res;
  gp.tokens = static_cast<uint32_t *>(d_tok);
  gp.bm = static_cast<uint32_t *>(d_bm);
  std::vector<GenResult> res(units);
  std::vector<GenLink> link(units);
  std::vector<uint32_t> todo(units), ltodo;
  for (size_t k = 0; k < units; ++k) todo[k] = (uint32_t)k;
  for (size_t k = 1; k < units; ++k) ltodo.push_back((uint32_t)k);
  ZT_HIP(hipMemcpyAsync(d_jobs, jobs.data(), units * sizeof(GenJob), hipMemcpyHostToDevice, s));
  // does end state `e` refute a guess whose source candidate is `src`?
  auto refutes = [](const GenState &e, const GenJob &j, uint64_t src) {
    if (src == ~0ull) return false;
    switch (j.st.kind) {
      case GK_HUFF: return !(e.kind == GK_HUFF && e.hdr == j.st.hdr);
      case GK_BLOCK: return !(e.kind == GK_BLOCK && e.pos == j.st.pos);
      case GK_SHDR: return !(e.kind == GK_SHDR && e.pos == j.st.pos);
      case GK_STORED: return !(e.kind == GK_STORED && e.pos == j.st.pos && e.rem == j.st.rem);
      default: return false;
    }
  };
  int pass = 0;
  size_t chain_end = 0;
  for (;; ++pass) {
    if (pass > 24) GFALLBACK("no convergence after %d passes\n", pass);
    // decode `todo`, link `ltodo`
    ZT_HIP(hipMemcpyAsync(d_which, todo.data(), todo.size() * 4, hipMemcpyHostToDevice, s));
    gp.which = d_which;
    gp.count = (uint32_t)todo.size();
    gen_tokenize_kernel<<<gp.count, 64, 0, s>>>(gp);
    ZT_HIP(hipGetLastError());
    if (!ltodo.empty()) {
      ZT_HIP(hipMemcpyAsync(d_lwhich, ltodo.data(), ltodo.size() * 4, hipMemcpyHostToDevice, s));
      gen_link_kernel<<<(uint32_t)ltodo.size(), 64, 0, s>>>(d_jobs, d_res, gp.bm, gp.tokens, d_lwhich, d_link);
      ZT_HIP(hipGetLastError());
    }
    {
      void *mb;
      const size_t rb = units * sizeof(GenResult), lb = units * sizeof(GenLink);
      ZT_TRY(mailbox(c, rb + lb, &mb));
      ZT_TRY(x_copy(mb, d_res, rb, s));
      ZT_TRY(x_copy((uint8_t *)mb + rb, d_link, lb, s));
      ZT_HIP(hipStreamSynchronize(s));
      memcpy(res.data(), mb, rb);
      memcpy(link.data(), (uint8_t *)mb + rb, lb);
    }
    // walk the chain (past broken units too: independent failures are all
    // redone in the same pass)
    std::vector<uint32_t> bad;
    bool ended = false, clean = true;
    for (size_t k = 0; k < units; ++k) {
      const bool linked = k == 0 || link[k].ok;
      if (!linked) {
        bad.push_back((uint32_t)k);
        clean = false;
      }
      if (clean && res[k].status != ZT_OK) GFALLBACK("unit %zu on the chain: status %d\n", k, res[k].status);
      if (res[k].end.kind == GK_FINAL && linked) {
        if (clean) {
          chain_end = k;
          ended = true;
        }
        break;
      }
    }
    if (gen_debug()) {
      fprintf(stderr, "[zt inflate gen] pass %d: %zu units, %u/%u candidates, %zu bad links\n", pass, units, nb, nc,
              bad.size());
      for (size_t q = 0; q < bad.size() && q < 3; ++q) {
        const size_t k = bad[q];
        const GenResult &a = res[k - 1], &b = res[k];
        const GenJob &j = jobs[k];
        fprintf(stderr,
                "  unit %zu job(kind %u pos %llu hdr %llu rem %u spec %u) | prev end(kind %u pos %llu hdr %llu rem %u "
                "fin %u) st %d tail %u | this st %d rec %u tab %llu fin %u dec %llu ntok %u\n",
                k, j.st.kind, (unsigned long long)j.st.pos, (unsigned long long)j.st.hdr, j.st.rem, j.spec,
                a.end.kind, (unsigned long long)a.end.pos, (unsigned long long)a.end.hdr, a.end.rem, a.end.bfinal,
                a.status, a.tail_ok, b.status, b.recorded, (unsigned long long)b.tab_id, b.tab_final,
                (unsigned long long)b.dec_start, b.ntok);
      }
    }
    if (bad.empty()) {
      if (!ended) GFALLBACK("the chain ends without a final block\n");
      break;
    }
    // redo the bad units from their predecessor's end; a guess the
    // predecessor's end refutes is replaced, in every later unit that made
    // it, by what that end state says about the stream there
    todo.clear();
    ltodo.clear();
    std::vector<uint8_t> mark(units, 0);
    std::vector<std::pair<uint64_t, uint32_t>> refuted;  // (source candidate, failing unit)
    for (uint32_t k : bad) {
      const GenResult &pr = res[k - 1];
      if (pr.status != ZT_OK || pr.end.kind == GK_FINAL) continue;
      GenJob &j = jobs[k];
      if (j.spec && refutes(pr.end, j, srcs[k])) refuted.push_back({srcs[k], k});
      j.st = pr.end;
      j.spec = 0;
      srcs[k] = ~0ull;
      mark[k] = 1;
    }
    if (!refuted.empty()) {
      std::sort(refuted.begin(), refuted.end());
      size_t w = 0;
      for (size_t i = 0; i < refuted.size(); ++i)
        if (i == 0 || refuted[i].first != refuted[i - 1].first) refuted[w++] = refuted[i];
      refuted.resize(w);
      for (size_t m = 1; m < units; ++m) {
        GenJob &jm = jobs[m];
        if (!jm.spec || mark[m]) continue;
        auto it = std::lower_bound(refuted.begin(), refuted.end(), std::make_pair(srcs[m], 0u));
        if (it == refuted.end() || it->first != srcs[m] || it->second >= m) continue;
        const GenState &e = res[it->second - 1].end;  // the state the chain showed there
        const uint64_t x = jm.st.pos;
        if (e.kind == GK_HUFF || e.kind == GK_BLOCK) {
          jm.st.kind = GK_HUFF;
          jm.st.hdr = e.kind == GK_HUFF ? e.hdr : e.pos;
          jm.st.bfinal = e.bfinal;
          srcs[m] = jm.st.hdr;
        } else if (e.kind == GK_STORED && x >= e.pos && x < e.pos + 8 * (uint64_t)e.rem && (x & 7) == 0) {
          jm.st.kind = GK_STORED;
          jm.st.rem = (uint32_t)(e.rem - (x - e.pos) / 8);
          jm.st.bfinal = e.bfinal;
          srcs[m] = e.pos;
        } else {
          continue;
        }
        mark[m] = 1;
      }
    }
    for (size_t k = 0; k < units; ++k)
      if (mark[k]) {
        todo.push_back((uint32_t)k);
        if (k > 0) ltodo.push_back((uint32_t)k);
        if (k + 1 < units && !mark[k + 1]) ltodo.push_back((uint32_t)(k + 1));
      }
    std::sort(ltodo.begin(), ltodo.end());
    ltodo.erase(std::unique(ltodo.begin(), ltodo.end()), ltodo.end());
    if (todo.empty()) GFALLBACK("failed links with no redo (pass %d)\n", pass);
    ZT_HIP(hipMemcpyAsync(d_jobs, jobs.data(), units * sizeof(GenJob), hipMemcpyHostToDevice, s));
  }
  if (gen_debug()) fprintf(stderr, "[zt inflate gen] %zu units, %u candidates, %d passes\n", units, nc, pass + 1);
  // ---- chain units and segments
  std::vector<ChainUnit> chain;
  std::vector<SegJob> segs;
  std::vector<GenSeg> gsegs;
  // copy segments: enough for two waves per CU, 128 KiB .. 1 MiB each
  uint64_t out_est = 0;
  for (size_t k = 0; k <= chain_end; ++k) out_est += res[k].out_stop;
  uint64_t kSeg = std::min<uint64_t>(
      1u << 20, std::max<uint64_t>(128u << 10, out_est / (2 * (uint64_t)std::max(c->num_cu, 1))));
  if (getenv("ZT_GEN_SEG")) kSeg = std::max<uint64_t>(64u << 10, (uint64_t)atoll(getenv("ZT_GEN_SEG")));
  uint64_t total = 0, seg_start = 0, desc_total = 0, desc_seg = 0, base16 = 0;
  for (size_t k = 0; k <= chain_end; ++k) {
    // unit k's tokens [t, cut): from its join with k-1 to its join with k+1
    const uint32_t t = k ? link[k].t : 0;
    const uint64_t by = k ? link[k].bytes : 0;
    const uint32_t cut = k < chain_end ? link[k + 1].prev_cut : res[k].ntok_stop;
    const uint64_t cb = k < chain_end ? link[k + 1].prev_bytes : res[k].out_stop;
    if (cut < t || cb < by) GFALLBACK("unit %zu: join order\n", k);
    const uint64_t ol = cb - by;
    if (ol > 0xFFFFFFFFull) GFALLBACK("unit %zu: %llu output bytes\n", k, (unsigned long long)ol);
    if (segs.empty() || total - seg_start >= kSeg) {
      if (!segs.empty()) {
        gsegs.back().len = total - seg_start;
        base16 += al256(total - seg_start);
      }
      desc_total = (desc_total + 511) & ~uint64_t(511);
      desc_seg = desc_total;
      seg_start = total;
      segs.push_back(SegJob{(uint32_t)chain.size(), 0});
      gsegs.push_back(GenSeg{base16, total, 0});
    }
    chain.push_back(ChainUnit{jobs[k].tok_off + t, total, seg_start, desc_seg + (total - seg_start), cut - t,
                              (uint32_t)ol});
    segs.back().count++;
    total += ol;
    desc_total = desc_seg + (total - seg_start);
  }
  gsegs.back().len = total - seg_start;
  base16 += al256(total - seg_start);
  if (gen_debug()) {
    fprintf(stderr, "[zt inflate gen] chain %zu units, %zu segments of ~%llu B, output %llu B\n", chain.size(),
            gsegs.size(), (unsigned long long)kSeg, (unsigned long long)total);
    if (getenv("ZT_GEN_TOKDUMP")) {
      const size_t k = (size_t)atoll(getenv("ZT_GEN_TOKDUMP"));
      for (size_t u = k - 1; u <= k && u < units; ++u) {
        std::vector<uint32_t> tk(res[u].ntok);
        ZT_HIP(hipMemcpy(tk.data(), gp.tokens + jobs[u].tok_off, tk.size() * 4, hipMemcpyDeviceToHost));
        fprintf(stderr, "TOK unit %zu ntok_stop %u ntok %u:", u, res[u].ntok_stop, res[u].ntok);
        const size_t a0 = u == k ? 0 : (res[u].ntok_stop > 20 ? res[u].ntok_stop - 20 : 0);
        for (size_t i = a0; i < tk.size() && i < a0 + 120; ++i) fprintf(stderr, " %zu:%x", i, tk[i]);
        fprintf(stderr, "\n");
      }
    }
    if (getenv("ZT_GEN_DUMP")) {
      for (size_t i = 0; i < chain.size(); ++i)
        fprintf(stderr,
                "  cu %zu out %llu len %u ntok %u | job kind %u pos %llu spec %u | t %u by %llu | cut %u cb %llu | "
                "dec %llu end %u@%llu ntok %u/%u out %llu/%llu\n",
                i, (unsigned long long)chain[i].out_off, chain[i].out_len, chain[i].ntok, jobs[i].st.kind,
                (unsigned long long)jobs[i].st.pos, jobs[i].spec, i ? link[i].t : 0,
                (unsigned long long)(i ? link[i].bytes : 0), i < chain_end ? link[i + 1].prev_cut : res[i].ntok_stop,
                (unsigned long long)(i < chain_end ? link[i + 1].prev_bytes : res[i].out_stop),
                (unsigned long long)res[i].dec_start, res[i].end.kind, (unsigned long long)res[i].end.pos,
                res[i].ntok_stop, res[i].ntok, (unsigned long long)res[i].out_stop,
                (unsigned long long)res[i].out_len);
      for (size_t i = 0; i < gsegs.size(); ++i)
        fprintf(stderr, "  seg %zu out %llu len %llu first %u count %u\n", i, (unsigned long long)gsegs[i].out_off,
                (unsigned long long)gsegs[i].len, segs[i].first, segs[i].count);
    }
  }
  *out_len = total;
  *end_ip = (res[chain_end].end.pos + 7) >> 3;
  uint8_t *d_out = *d_out_io;
  if (!d_out) {
    void *p;
    ZT_TRY(scratch(c, 1, total ? total : 1, &p));
    d_out = static_cast<uint8_t *>(p);
    *d_out_io = d_out;
  } else if (total > out_cap) {
    return set_error(ZT_E_ARG, "output capacity too small");
  }
  if (total == 0) return ZT_OK;
  // ---- 4. expand, copy with markers, windows, final bytes
  void *d_chain, *d_desc, *d_o16, *d_win;
  const size_t chain_bytes = al256(chain.size() * sizeof(ChainUnit));
  const size_t seg_bytes = al256(segs.size() * sizeof(SegJob));
  const size_t gseg_bytes = al256(gsegs.size() * sizeof(GenSeg));
  const size_t ust_bytes = al256(chain.size() * 4);
  ZT_TRY(scratch(c, 14, chain_bytes + seg_bytes + gseg_bytes + ust_bytes + al256(segs.size() * 4), &d_chain));
  ZT_TRY(scratch(c, 15, (desc_total + 1024) * 2, &d_desc));
  ZT_TRY(scratch(c, 16, (base16 + 256) * 2, &d_o16));
  ZT_TRY(scratch(c, 17, gsegs.size() * (size_t)RING, &d_win));
  uint8_t *cb = static_cast<uint8_t *>(d_chain);
  ChainUnit *d_cu = reinterpret_cast<ChainUnit *>(cb);
  SegJob *d_sj = reinterpret_cast<SegJob *>(cb + chain_bytes);
  GenSeg *d_gs = reinterpret_cast<GenSeg *>(cb + chain_bytes + seg_bytes);
  int32_t *d_ust = reinterpret_cast<int32_t *>(cb + chain_bytes + seg_bytes + gseg_bytes);
  int32_t *d_st = reinterpret_cast<int32_t *>(cb + chain_bytes + seg_bytes + gseg_bytes + ust_bytes);
  ZT_HIP(hipMemcpyAsync(d_cu, chain.data(), chain.size() * sizeof(ChainUnit), hipMemcpyHostToDevice, s));
  ZT_HIP(hipMemcpyAsync(d_sj, segs.data(), segs.size() * sizeof(SegJob), hipMemcpyHostToDevice, s));
  ZT_HIP(hipMemcpyAsync(d_gs, gsegs.data(), gsegs.size() * sizeof(GenSeg), hipMemcpyHostToDevice, s));
  ResolveParams rp;
  rp.tokens = gp.tokens;
  rp.units = d_cu;
  rp.segs = d_sj;
  rp.out = d_out;
  rp.desc = static_cast<uint16_t *>(d_desc);
  rp.unit_status = d_ust;
  rp.seg_status = d_st;
  rp.nunits = (uint32_t)chain.size();
  rp.nseg = (uint32_t)segs.size();
  rp.marker = 1;
  rp.in = nullptr;  // (the general tokenizer writes no run tokens)
  ZT_TRY(expand_units_dev(rp, s));
  uint16_t *o16 = static_cast<uint16_t *>(d_o16);
  copy_marker_kernel<<<rp.nseg, 64, 0, s>>>(rp, d_gs, o16);
  ZT_HIP(hipGetLastError());
  uint8_t *wins = static_cast<uint8_t *>(d_win);
  if (gsegs.size() > 1) {
    const uint32_t nwin = (uint32_t)gsegs.size() - 1;
    static const bool serial = getenv("ZT_GEN_WCHAIN") != nullptr;  // (A/B: the serial window chain)
    void *d_wj = nullptr;
    if (!serial && nwin < WJ_MAXWIN && scratch(c, 26, 2 * (size_t)nwin * RING * 4, &d_wj) == ZT_OK) {
      uint32_t *e0 = static_cast<uint32_t *>(d_wj), *e1 = e0 + (size_t)nwin * RING;
      const uint32_t grid = (uint32_t)(((uint64_t)nwin * RING / 4 + 255) / 256);
      wj_init_kernel<<<grid, 256, 0, s>>>(d_gs, nwin, o16, e0);
      ZT_HIP(hipGetLastError());
      int rounds = 1;
      while ((1u << (rounds - 1)) < nwin) ++rounds;  // ceil(log2 nwin) + 1
      for (int r = 0; r < rounds; ++r) {
        wj_round_kernel<<<grid, 256, 0, s>>>(e0, e1, nwin, r + 1 == rounds, wins, d_st);
        ZT_HIP(hipGetLastError());
        std::swap(e0, e1);
      }
    } else {
      (void)hipGetLastError();  // (a failed allocation's sticky error)
      window_chain_kernel<<<1, 1024, 0, s>>>(d_gs, nwin, o16, wins);
      ZT_HIP(hipGetLastError());
    }
  }
  uint64_t maxlen = 0;
  for (const GenSeg &g : gsegs) maxlen = std::max(maxlen, g.len);
  dim3 grid((uint32_t)((maxlen + 4095) / 4096), (uint32_t)gsegs.size());
  marker_resolve_kernel<<<grid, 256, 0, s>>>(d_gs, o16, wins, d_out);
  ZT_HIP(hipGetLastError());
  ZT_TRY(timing_end(c, s, 2));
  std::vector<int32_t> ust(chain.size()), sst(segs.size());
  {
    void *mb;
    ZT_TRY(mailbox(c, (chain.size() + segs.size()) * 4, &mb));
    ZT_TRY(x_copy(mb, d_ust, chain.size() * 4, s));
    ZT_TRY(x_copy((uint8_t *)mb + chain.size() * 4, d_st, segs.size() * 4, s));
    ZT_HIP(hipStreamSynchronize(s));
    memcpy(ust.data(), mb, chain.size() * 4);
    memcpy(sst.data(), (uint8_t *)mb + chain.size() * 4, segs.size() * 4);
  }
  ZT_TRY(timing_collect(c, &c->times.inflate_ms, &c->times.inflate_launches, 2));
  for (size_t i = 0; i < chain.size(); ++i)
    if (ust[i] != ZT_OK) GFALLBACK("chain unit %zu: status %d\n", i, ust[i]);
  for (size_t i = 0; i < segs.size(); ++i)
    if (sst[i] != ZT_OK) GFALLBACK("segment %zu: status %d\n", i, sst[i]);
  c->times.inflate_paths[1]++;
  c->times.general_passes += (uint64_t)pass + 1;
  return ZT_OK;
}

}  // namespace zt
