// inflate_common.h -- device pieces shared by the one-wave inflate (inflate.hip)
// and the two-phase token inflate (inflate_tok.hip): canonical Huffman decode
// tables in LDS, the LDS-staged bit reader, and the block-header parser.
// Follows src/RawInflate.ts:145-400 and src/Huffman.ts:8-68.
#pragma once
#include "zt_internal.h"

namespace zt {
namespace {


constexpr int RING = 32768;
constexpr uint32_t RING_MASK = RING - 1;
constexpr int GRAN = 16384;  // output flush granule (ring holds 32 KiB of history)
#ifndef ZT_PRI
#define ZT_PRI 8
#endif
constexpr int PRI = ZT_PRI;

// PRI: primary table bits.  8 (1 KiB per table): every 8-bit code -- all
// literals of the reference's blocks over random bytes -- decodes from one
// lookup instead of the canonical search's three dependent LDS reads
// (tokenize of the C2 batch 15.5 -> 11.5 ms, bench 4.05 -> 3.94 ms per GiB;
// profiles/r04pri_*).  tokenize_kernel's 12.5 KiB of LDS still allows the
// 12 units per CU its registers allow (3 waves per SIMD).  Round 1 chose 7
// over 8..10 when LDS, not registers, set the units per CU.
// Primary-table entry (u32): bits 0-3 code length (0 = code longer than PRI
// bits: canonical search), 4-7 extra bits, 8-16 symbol, 17-31 base value
// (match length for literal/length symbols > 256, distance for distance
// symbols < 30).
struct HuffTab {
  uint32_t pri[1 << PRI];
  uint16_t sorted[320];
  uint32_t first[16];
  uint32_t count[16];
  uint32_t offs[16];
  uint32_t running[16];
  uint64_t lim[16];   // (first + count) << (32 - l): left-justified end of the length-l codes
  int32_t base[16];   // offs - first: sorted[] index of a code of length l is base + code
  int maxlen;
  int status;
};


__device__ __forceinline__ uint32_t uni(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ uint64_t uni64(uint64_t v) {
  return ((uint64_t)uni((uint32_t)(v >> 32)) << 32) | uni((uint32_t)v);
}
// One wavefront per workgroup: LDS operations of a wave execute in order, so
// cross-lane LDS hand-offs only need the compiler not to reorder.  (A
// __syncthreads() here would also wait for every outstanding global load and
// store -- the input prefetch and the output flushes.)
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_wave_barrier();
  asm volatile("" ::: "memory");
}

__device__ __forceinline__ uint64_t lanemask_lt(int lane) { return (lane == 0) ? 0ull : (~0ull >> (64 - lane)); }

// Build a canonical decode table from `n` code lengths in s->lens[off..off+n).
// Returns 0, or ZT_E_BAD_TREE for an over-subscribed length set.
__device__ __forceinline__ int build_table(const uint8_t *lens, int n, HuffTab *t, int lane, bool is_dist) {
  if (lane < 16) {
    t->count[lane] = 0;
    t->running[lane] = 0;
  }
  wave_sync();
  for (int s = lane; s < n; s += 64) {
    int l = lens[s];
    if (l) atomicAdd(&t->count[l], 1u);
  }
  wave_sync();
  if (lane == 0) {
    uint32_t code = 0, off = 0;
    int left = 1, maxlen = 0, st = 0;
    t->count[0] = 0;
    for (int l = 1; l < 16; ++l) {
      code = (code + t->count[l - 1]) << 1;
      t->first[l] = code;
      t->offs[l] = off;
      off += t->count[l];
      left = (left << 1) - (int)t->count[l];
      if (left < 0) st = ZT_E_BAD_TREE;
      if (t->count[l]) maxlen = l;
    }
    t->first[0] = 0;
    t->offs[0] = 0;
    for (int l = 1; l < 16; ++l) {
      t->lim[l] = (uint64_t)(t->first[l] + t->count[l]) << (32 - l);
      t->base[l] = (int32_t)t->offs[l] - (int32_t)t->first[l];
    }
    t->maxlen = maxlen;
    t->status = st;
  }
  wave_sync();
  // symbols sorted by (length, symbol): rank among equal lengths via ballots
  for (int base = 0; base < n; base += 64) {
    int s = base + lane;
    int l = s < n ? lens[s] : 0;
    uint64_t peers = 0;
#pragma unroll
    for (int L = 1; L < 16; ++L) {
      uint64_t m = __ballot(l == L);
      if (l == L) peers = m;
    }
    uint32_t below = __popcll(peers & lanemask_lt(lane));
    if (l) t->sorted[t->offs[l] + t->running[l] + below] = (uint16_t)s;
    wave_sync();
    if (l && below == 0) t->running[l] += __popcll(peers);
    wave_sync();
  }
  // primary table: entry e decodes the code whose bits (first bit = bit 0 of e)
  // are a prefix of e
  const int ml = t->maxlen < PRI ? t->maxlen : PRI;
  for (int e = lane; e < (1 << PRI); e += 64) {
    uint32_t r = __brev((uint32_t)e);
    uint32_t ent = 0;
    for (int l = 1; l <= ml; ++l) {
      uint32_t c = r >> (32 - l);
      uint32_t k = c - t->first[l];
      if (k < t->count[l]) {
        const uint32_t sym = t->sorted[t->offs[l] + k];
        uint32_t ex = 0, base = 0;
        if (is_dist) {
          if (sym < 30) {
            ex = dist_extra(sym);
            base = dist_base(sym);
          }
        } else if (sym > 256) {  // 286/287 decode as length 258, like the reference
          ex = len_extra(sym - 257);
          base = len_base(sym - 257);
        }
        ent = (uint32_t)l | (ex << 4) | (sym << 8) | (base << 17);
        break;
      }
    }
    t->pri[e] = ent;
  }
  wave_sync();
  return t->status;
}

// Input bits: the compressed stream is staged through an IN_RING-byte LDS
// ring by cooperative half-ring refills (one wait per half ring of input,
// never inside the per-symbol chain); a 64-bit bit buffer in scalar registers
// is topped up from LDS.  Positions are relative to a 16-byte aligned base
// below `in`.  4 KiB (not 8) keeps tokenize_kernel at 18.5 KiB of LDS: 8
// units per CU instead of 6 (tokenize 7.1 -> 5.9 ms per GiB).
#ifndef ZT_IN_RING
#define ZT_IN_RING 4096
#endif
constexpr uint32_t IN_RING = ZT_IN_RING;
constexpr uint32_t IN_RING_WORDS = IN_RING / 4;
constexpr uint32_t IN_HALF = IN_RING / 2;
constexpr uint32_t IN_MASK_W = IN_RING / 4 - 1;

// load IN_HALF bytes [fill, fill + IN_HALF) into the ring (all lanes).  Out
// of line and by value, so the reader state stays in registers and the global
// loads (and their waits) stay off the symbol loop.
__device__ __attribute__((noinline)) void refill_half_ring(g_u8 *abase, uint32_t *inbuf, uint64_t lo, uint64_t hi,
                                                           uint64_t fill, int lane) {
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  typedef __attribute__((address_space(1))) const u32x4 g_u32x4;
  typedef __attribute__((address_space(3))) uint32_t l_u32;
  l_u32 *lb = (l_u32 *)inbuf;
  for (uint32_t k = 0; k < IN_HALF / 1024; ++k) {
    const uint64_t off = fill + (uint64_t)k * 1024 + (uint64_t)lane * 16;
    u32x4 v = {0, 0, 0, 0};
    if (off < hi) v = *(g_u32x4 *)(abase + off);
    if (off < lo || off + 16 > hi) {
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        const uint64_t b = off + j;
        if (b < lo || b >= hi) v[j >> 2] &= ~(0xFFu << (8 * (j & 3)));
      }
    }
    const uint32_t wi = (uint32_t)((off >> 2) & IN_MASK_W);
    lb[wi] = v.x;
    lb[wi + 1] = v.y;
    lb[wi + 2] = v.z;
    lb[wi + 3] = v.w;
    if (wi == 0) {  // mirror of the ring start
      lb[IN_RING / 4] = v.x;
      lb[IN_RING / 4 + 1] = v.y;
      lb[IN_RING / 4 + 2] = v.z;
      lb[IN_RING / 4 + 3] = v.w;
    }
  }
  wave_sync();
}

struct Reader {
  g_u8 *abase;          // 16-B aligned base
  uint32_t *inbuf;      // LDS ring (IN_RING bytes + 16 mirror bytes)
  uint64_t lo, hi;      // valid input bytes are [lo, hi) (relative to abase)
  uint64_t fill;        // ring holds bytes [fill - IN_RING, fill)
  uint64_t ip;          // next byte to shift into bb
  uint64_t bb;          // bit buffer (LSB = next bit)
  uint32_t bc;          // valid bits in bb
  uint64_t ip_ref;      // reference's ip (strict mode), relative to `in`
  int strict_fail;
  int lane;

  __device__ __forceinline__ void refill_half() {
    refill_half_ring(abase, inbuf, lo, hi, fill, lane);
    fill += IN_HALF;
  }
  __device__ void init(const uint8_t *p, uint64_t n, uint64_t start, uint32_t *buf, int ln) {
    lane = ln;
    inbuf = buf;
    uintptr_t a = reinterpret_cast<uintptr_t>(p);
    abase = (g_u8 *)(a & ~uintptr_t(15));
    lo = a & 15;
    hi = lo + n;
    ip = lo + start;
    fill = ip & ~uint64_t(IN_HALF - 1);
    refill_half();
    refill_half();
    bb = 0;
    bc = 0;
    ip_ref = start;
    strict_fail = 0;
  }
  // 8 bytes at ring position q (mirror covers the wrap)
  __device__ __forceinline__ uint64_t ld64(uint64_t q) const {
    const uint32_t w = (uint32_t)((q >> 2) & IN_MASK_W);
    const uint32_t sh = (uint32_t)(q & 3);
    const uint32_t a = inbuf[w], b = inbuf[w + 1], c = inbuf[w + 2];
    const uint32_t x = __builtin_amdgcn_alignbyte(b, a, sh);
    const uint32_t y = __builtin_amdgcn_alignbyte(c, b, sh);
    return ((uint64_t)uni(y) << 32) | uni(x);
  }
  // keep >= 56 valid bits in bb (bits past the end read as 0)
  __device__ __forceinline__ void refill() {
    if (bc <= 56) {
      if (ip + 8 > fill - IN_HALF + IN_HALF && ip + 16 > fill) refill_half();
      bb |= ld64(ip) << bc;
      ip += (63 - bc) >> 3;
      bc |= 56;
    }
  }
  // consumed bits, relative to the aligned base
  __device__ __forceinline__ uint64_t pos_bits() const { return ip * 8 - bc; }
  __device__ __forceinline__ uint64_t pos_bits_in() const { return pos_bits() - lo * 8; }  // relative to `in`
  __device__ __forceinline__ bool past_end(uint32_t extra) const { return pos_bits() + extra > hi * 8; }
  // readBits(nb) with the reference's EOF test (strict) and the RFC bound
  template <bool STRICT>
  __device__ __forceinline__ bool bits(int nb, uint32_t &out) {
    const uint64_t bp = pos_bits_in();
    if (STRICT) {
      int64_t bbl = (int64_t)(ip_ref * 8) - (int64_t)bp;
      int64_t need = ((int64_t)nb - bbl + 7) >> 3;
      if ((int64_t)ip_ref + need >= (int64_t)(hi - lo)) {
        strict_fail = 1;
        return false;
      }
      uint64_t want = (bp + nb + 7) >> 3;
      if (want > ip_ref) ip_ref = want;
    }
    if (past_end(nb)) return false;
    refill();
    out = (uint32_t)bb & ((1u << nb) - 1);
    bb >>= nb;
    bc -= nb;
    return true;
  }
  __device__ __forceinline__ void code_refill(int maxlen) {
    uint64_t want = (pos_bits_in() + maxlen + 7) >> 3;
    if (want > hi - lo) want = hi - lo;
    if (want > ip_ref) ip_ref = want;
  }
  // jump to bit position pb (relative to abase), reloading the ring
  __device__ void seek_bit(uint64_t pb) {
    const uint64_t a = pb >> 3;
    bb = 0;
    bc = 0;
    ip = a;
    fill = a & ~uint64_t(IN_HALF - 1);
    refill_half();
    refill_half();
    refill();
    const uint32_t drop = (uint32_t)(pb & 7);
    bb >>= drop;
    bc -= drop;
  }
  // jump to a byte position relative to `in` (stored blocks)
  __device__ void seek_byte(uint64_t p) {
    const uint64_t a = p + lo;
    bb = 0;
    bc = 0;
    ip = a;
    if (a + 16 > fill || a < fill - IN_RING) {
      fill = a & ~uint64_t(IN_HALF - 1);
      refill_half();
      refill_half();
    }
  }
};

// Decode one symbol; returns symbol or a negative status; *clen = code length
template <bool STRICT>
__device__ __forceinline__ int decode_sym(Reader &rd, const HuffTab *t, int &clen) {
  if (STRICT) rd.code_refill(t->maxlen);
  rd.refill();
  const uint32_t v = (uint32_t)rd.bb;
  uint32_t e = uni(t->pri[v & ((1u << PRI) - 1)]);
  int len, sym;
  if (e & 15) {
    len = (int)(e & 15);
    sym = (int)((e >> 8) & 511);
  } else {
    // canonical limits (see HuffTab::lim): the length is one more than the
    // number of lengths whose code range ends at or below the peek
    const uint64_t r = __brev(v);
    uint32_t l = PRI + 1;
#pragma unroll
    for (int k = PRI + 1; k < 16; ++k) l += r >= t->lim[k] ? 1u : 0u;
    l = uni(l);
    if (l > (uint32_t)uni((uint32_t)t->maxlen)) return ZT_E_INVALID_SYMBOL;  // bits match no code of an incomplete set
    len = (int)l;
    sym = (int)uni(t->sorted[t->base[l] + (int32_t)((uint32_t)r >> (32 - l))]);
  }
  clen = len;
  if (rd.past_end((uint32_t)len)) return ZT_E_INVALID_CODE_LENGTH;
  rd.bb >>= len;
  rd.bc -= len;
  return sym;
}

__constant__ uint8_t kClOrder[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

// Decode tables of a BTYPE 1 / 2 block (fixed codes, or the dynamic header of
// src/RawInflate.ts:345-400) into lt / dt; `lens` is >= 320 bytes of LDS.
// Returns 0 or a status (detail: code length / BTYPE for the message).
template <bool STRICT>
__device__ int read_tables(Reader &rd, uint8_t *lens, HuffTab *lt, HuffTab *dt, uint32_t btype, int lane,
                           int &detail) {
  uint32_t v;
  if (btype == 1) {
    // fixed tables (RFC 1951 3.2.6)
    for (int s = lane; s < 288; s += 64) lens[s] = s <= 143 ? 8 : s <= 255 ? 9 : s <= 279 ? 7 : 8;
    wave_sync();
    build_table(lens, 288, lt, lane, false);
    for (int s = lane; s < 30; s += 64) lens[s] = 5;
    wave_sync();
    build_table(lens, 30, dt, lane, true);
    return ZT_OK;
  }
  if (btype != 2) {
    detail = (int)btype;
    return ZT_E_UNKNOWN_BTYPE;
  }
  uint32_t hlit, hdist, hclen;
  if (!rd.template bits<STRICT>(5, hlit) || !rd.template bits<STRICT>(5, hdist) ||
      !rd.template bits<STRICT>(4, hclen))
    return ZT_E_INPUT_BROKEN;
  hlit += 257;
  hdist += 1;
  hclen += 4;
  if (lane < 19) lens[lane] = 0;
  wave_sync();
  bool ok = true;
  for (uint32_t i = 0; i < hclen; ++i) {
    if (!rd.template bits<STRICT>(3, v)) {
      ok = false;
      break;
    }
    if (lane == 0) lens[kClOrder[i]] = (uint8_t)v;
  }
  wave_sync();
  if (!ok) return ZT_E_INPUT_BROKEN;
  int bst = build_table(lens, 19, dt, lane, false);  // code-length code lives in `dt` for now
  if (bst) return bst;
  const uint32_t total = hlit + hdist;
  for (int s = lane; s < 320; s += 64) lens[s] = 0;
  wave_sync();
  uint32_t i = 0, prev = 0;
  int status = ZT_OK;
  while (i < total) {
    int clen;
    int sym = decode_sym<STRICT>(rd, dt, clen);
    if (sym < 0) {
      status = sym;
      detail = clen;
      break;
    }
    uint32_t rep, val;
    if (sym == 16) {
      if (!rd.template bits<STRICT>(2, v)) { status = ZT_E_INPUT_BROKEN; break; }
      rep = 3 + v;
      val = prev;
    } else if (sym == 17) {
      if (!rd.template bits<STRICT>(3, v)) { status = ZT_E_INPUT_BROKEN; break; }
      rep = 3 + v;
      val = 0;
      prev = 0;
    } else if (sym == 18) {
      if (!rd.template bits<STRICT>(7, v)) { status = ZT_E_INPUT_BROKEN; break; }
      rep = 11 + v;
      val = 0;
      prev = 0;
    } else {
      rep = 1;
      val = (uint32_t)sym;
      prev = val;
    }
    // writes past hlit+hdist are dropped, as into the reference's Uint8Array
    for (uint32_t k = lane; k < rep; k += 64)
      if (i + k < total) lens[i + k] = (uint8_t)val;
    i += rep;
  }
  wave_sync();
  if (status) return status;
  bst = build_table(lens, (int)hlit, lt, lane, false);
  if (!bst) bst = build_table(lens + hlit, (int)hdist, dt, lane, true);
  return bst;
}

}  // namespace
}  // namespace zt
