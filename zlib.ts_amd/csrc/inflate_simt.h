// inflate_simt.h -- Huffman block bodies to tokens, shared by the sync-point
// tokenizer (inflate_tok.hip) and the general speculative tokenizer
// (inflate_gen.hip): the lane-uniform scalar decoder and the 64-lane
// speculative (SIMT) decoder.  Follows src/RawInflate.ts:466-516.
#pragma once
#include "inflate_common.h"

namespace zt {
namespace {

// token staging: lane k of `stg` holds token (ntok & ~63) + k of the current
// group of 64; a full group is written with one coalesced 256-byte store
struct TokOut {
  uint32_t *tok;
  uint32_t cap;
  uint32_t ntok;
  uint32_t stg;
  int lane;

  __device__ __forceinline__ void emit(uint32_t t) {
    const uint32_t k = uni(ntok);
    if (lane == (int)(k & 63)) stg = t;
    ntok = k + 1;
    if (((k + 1) & 63) == 0) tok[k - 63 + lane] = stg;
  }
  __device__ __forceinline__ void flush_partial() {
    const uint32_t c = ntok & 63;
    if (lane < (int)c) tok[(ntok & ~63u) + lane] = stg;
  }
};

// code longer than PRI bits: canonical search (src/Huffman.ts semantics)
__device__ __forceinline__ int long_code(const HuffTab *t, uint32_t v, uint32_t &len) {
  const uint32_t r = __brev(v);
  const int ml = (int)uni((uint32_t)t->maxlen);
  for (int l = PRI + 1; l <= ml; ++l) {
    const uint32_t c = r >> (32 - l);
    const uint32_t k = c - uni(t->first[l]);
    if (k < uni(t->count[l])) {
      len = (uint32_t)l;
      return (int)uni(t->sorted[uni(t->offs[l]) + k]);
    }
  }
  return -1;
}

// Huffman block body -> tokens (non-strict reader).  Returns 0 at end of
// block, or a status.
__device__ __forceinline__ int tok_huffman(Reader &rd, const HuffTab *lt, const HuffTab *dt, TokOut &to,
                                           uint64_t &op) {
  const uint64_t hib = uni64(rd.hi) * 8;
  constexpr uint32_t M = (1u << PRI) - 1;
  for (;;) {
    rd.refill();  // >= 56 valid bits: one token needs at most 15 + 5 + 15 + 13
    const uint64_t bb = uni64(rd.bb);
    const uint32_t e = uni(lt->pri[(uint32_t)bb & M]);
    uint32_t cl, sym, ex, base;
    if (e & 15) {
      cl = e & 15;
      sym = (e >> 8) & 511;
      ex = (e >> 4) & 15;
      base = e >> 17;
    } else {
      const int s = long_code(lt, (uint32_t)bb, cl);
      if (s < 0) return ZT_E_INVALID_SYMBOL;
      sym = (uint32_t)s;
      ex = sym > 256 ? len_extra(sym - 257) : 0;
      base = sym > 256 ? len_base(sym - 257) : 0;
    }
    if (sym < 256) {
      if (to.ntok >= to.cap) return ZT_E_NOMEM;
      rd.bb = bb >> cl;
      rd.bc -= cl;
      to.emit(sym);
      op += 1;
      if (rd.pos_bits() > hib) return ZT_E_INPUT_BROKEN;
      continue;
    }
    if (sym == 256) {
      rd.bb = bb >> cl;
      rd.bc -= cl;
      if (rd.pos_bits() > hib) return ZT_E_INPUT_BROKEN;
      return ZT_OK;
    }
    const uint32_t length = base + ((uint32_t)(bb >> cl) & ((1u << ex) - 1));
    uint32_t used = cl + ex;
    const uint64_t b2 = bb >> used;
    const uint32_t d = uni(dt->pri[(uint32_t)b2 & M]);
    uint32_t dcl, dsym, dex, dbase;
    if (d & 15) {
      dcl = d & 15;
      dsym = (d >> 8) & 511;
      dex = (d >> 4) & 15;
      dbase = d >> 17;
    } else {
      const int s = long_code(dt, (uint32_t)b2, dcl);
      if (s < 0) return ZT_E_INVALID_SYMBOL;
      dsym = (uint32_t)s;
      dex = dsym < 30 ? dist_extra(dsym) : 0;
      dbase = dsym < 30 ? dist_base(dsym) : 0;
    }
    if (dsym >= 30) return ZT_E_INVALID_SYMBOL;
    const uint32_t dist = dbase + ((uint32_t)(b2 >> dcl) & ((1u << dex) - 1));
    used += dcl + dex;
    rd.bb = bb >> used;
    rd.bc -= used;
    if (rd.pos_bits() > hib) return ZT_E_INPUT_BROKEN;
    if (to.ntok >= to.cap) return ZT_E_NOMEM;
    to.emit((length << 16) | dist);
    op += length;
  }
}


// ------------------------------------------------ phase A, SIMT block body
// A Huffman block body is decoded by all 64 lanes at once, in rounds of
// 64 x SP_LANE_BITS bits, each lane from its own bit offset (speculative
// parallel decoding of a prefix code).  Lane l starts at s_l and decodes until
// it passes s_{l+1}, marking in a bitmap every position where a token began.
// Decoding is deterministic, so once a lane's path meets the true token
// sequence it *is* the true sequence.  The true start of lane l is the end of
// lane l-1's true path; if that position is marked in lane l's bitmap, lane l
// is synchronised and its tokens are the marks from there on (popcount).
// DEFLATE token streams often take tens of tokens to resynchronise (extra
// bits are raw), so unsynchronised lanes are re-decoded in parallel from
// their true start until they merge with their old path (a marked position),
// and the marks are corrected on the way.  A second pass decodes every lane's
// exact range and writes its tokens at their final index.
#ifndef ZT_SP_LANE_BITS
#define ZT_SP_LANE_BITS 448  // 416 / 448 / 480: tokenize 3.78 / 3.41 / 3.48 ms per GiB with the per-lane first pass (gpurun_out/r05bb)
#endif
constexpr uint32_t SP_LANE_BITS = ZT_SP_LANE_BITS;        // 56 bytes per lane
constexpr uint32_t SP_WORDS = SP_LANE_BITS / 32;          // bitmap words per lane
constexpr uint32_t SP_STAGE_BYTES = IN_RING;              // staged input per round
static_assert(64 * SP_LANE_BITS / 8 + 16 + 64 <= SP_STAGE_BYTES, "round must fit the stage");
static_assert(SP_STAGE_BYTES <= 4 * IN_RING_WORDS, "stage lives in the reader's ring");

struct SpecShared {
  uint32_t bm[SP_WORDS][64];  // token-start bitmap, word w of lane l
  uint32_t tail[64];          // the unit's last partial token group (staging)
};

// per-lane bit reader over the round's staged input (LDS, dword q at
// stage[q - qbase])
struct LaneBits {
  const uint32_t *stage;
  uint32_t qbase;
  uint32_t q;      // next dword to shift in
  uint32_t nw;     // that dword, read ahead: a refill is register work, off the
                   // token chain's LDS round trips (the read for the next one
                   // is issued before the token's table read)
  uint64_t bb;
  uint32_t bc;
  uint32_t rel;    // bit position of bb bit 0, relative to the body start

  __device__ __forceinline__ uint32_t word(uint32_t qq) const {
    return stage[(qq - qbase) & (SP_STAGE_BYTES / 4 - 1)];
  }
  // abs_bit: relative to the reader's abase; rel0: the same, relative to the body
  __device__ __forceinline__ void init(uint64_t abs_bit, uint32_t rel0) {
    q = (uint32_t)(abs_bit >> 5);
    const uint32_t sh = (uint32_t)abs_bit & 31;
    const uint32_t w0 = word(q), w1 = word(q + 1);
    nw = word(q + 2);
    bb = ((((uint64_t)w1) << 32) | w0) >> sh;
    bc = 64 - sh;
    q += 2;
    rel = rel0;
  }
  // afterwards at least 32 valid bits
  __device__ __forceinline__ void refill() {
    if (bc <= 32) {
      bb |= (uint64_t)nw << bc;
      bc += 32;
      ++q;
      nw = word(q);
    }
  }
  __device__ __forceinline__ void consume(uint32_t n) {
    bb >>= n;
    bc -= n;
    rel += n;
  }
};

// code longer than PRI bits, per lane
// (canonical limits: the length is one more than the number of lengths
// whose left-justified code range ends at or below the peek; all limits are
// read at once instead of a length-by-length search)
__device__ __forceinline__ int long_code_lane(const HuffTab *t, uint32_t v, uint32_t &len) {
  const uint64_t r = __brev(v);
  uint32_t l = PRI + 1;
#pragma unroll
  for (int k = PRI + 1; k < 16; ++k) l += r >= t->lim[k] ? 1u : 0u;
  if (l > (uint32_t)t->maxlen) return -1;
  len = l;
  return (int)t->sorted[t->base[l] + (int32_t)((uint32_t)r >> (32 - l))];
}

// one token at the lane's position: 0 ok (tok, nbytes), 1 end of block, -1 invalid
__device__ __forceinline__ int lane_token(LaneBits &lb, const HuffTab *lt, const HuffTab *dt, uint32_t &tok,
                                          uint32_t &nbytes) {
  constexpr uint32_t M = (1u << PRI) - 1;
  lb.refill();
  const uint32_t e = lt->pri[(uint32_t)lb.bb & M];
  uint32_t cl, sym, ex, base;
  if (e & 15) {
    cl = e & 15;
    sym = (e >> 8) & 511;
    ex = (e >> 4) & 15;
    base = e >> 17;
  } else {
    const int s = long_code_lane(lt, (uint32_t)lb.bb, cl);
    if (s < 0) return -1;
    sym = (uint32_t)s;
    ex = sym > 256 ? len_extra(sym - 257) : 0;
    base = sym > 256 ? len_base(sym - 257) : 0;
  }
  if (sym < 256) {
    lb.consume(cl);
    tok = sym;
    nbytes = 1;
    return 0;
  }
  if (sym == 256) {
    lb.consume(cl);
    return 1;
  }
  const uint32_t length = base + ((uint32_t)(lb.bb >> cl) & ((1u << ex) - 1));
  lb.consume(cl + ex);
  lb.refill();
  const uint32_t d = dt->pri[(uint32_t)lb.bb & M];
  uint32_t dcl, dsym, dex, dbase;
  if (d & 15) {
    dcl = d & 15;
    dsym = (d >> 8) & 511;
    dex = (d >> 4) & 15;
    dbase = d >> 17;
  } else {
    const int s = long_code_lane(dt, (uint32_t)lb.bb, dcl);
    if (s < 0) return -1;
    dsym = (uint32_t)s;
    dex = dsym < 30 ? dist_extra(dsym) : 0;
    dbase = dsym < 30 ? dist_base(dsym) : 0;
  }
  if (dsym >= 30) return -1;
  const uint32_t dist = dbase + ((uint32_t)(lb.bb >> dcl) & ((1u << dex) - 1));
  lb.consume(dcl + dex);
  tok = (length << 16) | dist;
  nbytes = length;
  return 0;
}

// lane_token for the first pass and the repairs: the token's bits consumed,
// its value not formed (same outcomes and bit positions)
__device__ __forceinline__ int lane_skip(LaneBits &lb, const HuffTab *lt, const HuffTab *dt) {
  constexpr uint32_t M = (1u << PRI) - 1;
  lb.refill();
  const uint32_t e = lt->pri[(uint32_t)lb.bb & M];
  uint32_t cl, sym, ex;
  if (e & 15) {
    cl = e & 15;
    sym = (e >> 8) & 511;
    ex = (e >> 4) & 15;
  } else {
    const int s = long_code_lane(lt, (uint32_t)lb.bb, cl);
    if (s < 0) return -1;
    sym = (uint32_t)s;
    ex = sym > 256 ? len_extra(sym - 257) : 0;
  }
  if (sym <= 256) {
    lb.consume(cl);
    return sym == 256 ? 1 : 0;
  }
  lb.consume(cl + ex);
  lb.refill();
  const uint32_t d = dt->pri[(uint32_t)lb.bb & M];
  uint32_t dcl, dsym, dex;
  if (d & 15) {
    dcl = d & 15;
    dsym = (d >> 8) & 511;
    dex = (d >> 4) & 15;
  } else {
    const int s = long_code_lane(dt, (uint32_t)lb.bb, dcl);
    if (s < 0) return -1;
    dsym = (uint32_t)s;
    dex = dsym < 30 ? dist_extra(dsym) : 0;
  }
  if (dsym >= 30) return -1;
  lb.consume(dcl + dex);
  return 0;
}

// the token that starts at bit abs_bit of the round's staged input, decoded on
// its own (its start is known: no reader state): all three words it can span
// are read at once, so several such decodes overlap their LDS round trips.
// Only called at a marked token start before the block's end code.
__device__ __forceinline__ void token_at(const uint32_t *stage, uint32_t qbase, uint64_t abs_bit, const HuffTab *lt,
                                         const HuffTab *dt, uint32_t &tok, uint32_t &nbytes) {
  constexpr uint32_t M = (1u << PRI) - 1;
  constexpr uint32_t QM = SP_STAGE_BYTES / 4 - 1;
  const uint32_t q = (uint32_t)(abs_bit >> 5), sh = (uint32_t)abs_bit & 31;
  const uint32_t w0 = stage[(q - qbase) & QM], w1 = stage[(q + 1 - qbase) & QM], w2 = stage[(q + 2 - qbase) & QM];
  const uint64_t lo = ((uint64_t)w1 << 32) | w0;
  uint64_t bb = sh ? (lo >> sh) | ((uint64_t)w2 << (64 - sh)) : lo;  // 64 valid bits
  const uint32_t e = lt->pri[(uint32_t)bb & M];
  uint32_t cl, sym, ex, base;
  if (e & 15) {
    cl = e & 15;
    sym = (e >> 8) & 511;
    ex = (e >> 4) & 15;
    base = e >> 17;
  } else {
    const int s = long_code_lane(lt, (uint32_t)bb, cl);
    sym = s < 0 ? 0u : (uint32_t)s;
    ex = sym > 256 ? len_extra(sym - 257) : 0;
    base = sym > 256 ? len_base(sym - 257) : 0;
  }
  if (sym < 256) {
    tok = sym;
    nbytes = 1;
    return;
  }
  const uint32_t length = base + ((uint32_t)(bb >> cl) & ((1u << ex) - 1));
  bb >>= cl + ex;
  const uint32_t d = dt->pri[(uint32_t)bb & M];
  uint32_t dcl, dsym, dex, dbase;
  if (d & 15) {
    dcl = d & 15;
    dsym = (d >> 8) & 511;
    dex = (d >> 4) & 15;
    dbase = d >> 17;
  } else {
    const int s = long_code_lane(dt, (uint32_t)bb, dcl);
    dsym = s < 0 ? 0u : (uint32_t)s;
    dex = dsym < 30 ? dist_extra(dsym) : 0;
    dbase = dsym < 30 ? dist_base(dsym) : 0;
  }
  tok = (length << 16) | (dbase + ((uint32_t)(bb >> dcl) & ((1u << dex) - 1)));
  nbytes = length;
}

// lane l-1's value (lane 0: `first`), with every lane taking part (DPP wave_shr:1)
__device__ __forceinline__ uint32_t from_prev_lane(uint32_t v, uint32_t first) {
  return (uint32_t)__builtin_amdgcn_update_dpp((int)first, (int)v, 0x138, 0xF, 0xF, false);
}

// ---- phase maps: blocks whose literal / length code is nearly fixed-length
// (the reference's single block over random bytes: ~8-bit codes) do not
// resynchronise -- a decode started off a token boundary stays off it, and
// the repairs above fix one lane per iteration.  For such blocks every lane
// instead maps each start phase x = 0..14 (bits past s_l) to the phase at
// which that decode crosses into the next lane's range (15: it ends the
// block, breaks, or crosses 15 or more bits past it); a prefix composition
// over the lanes gives every lane's true start at once.
#ifndef ZT_NO_PHASE_MAPS
__device__ __forceinline__ bool near_fixed_code(const HuffTab *lt) {
  // >= 90 % of the code space at one length
  uint32_t mx = 0;
#pragma unroll
  for (int k = 1; k < 16; ++k) {
    const uint32_t m = lt->count[k] << (15 - k);
    mx = m > mx ? m : mx;
  }
  return mx >= 29491u;
}

#ifndef ZT_PM_N
#define ZT_PM_N 3  // 161 VGPRs (3 waves per SIMD); C2 tokenize 5.20 / 5.23 / 5.33 ms with 3 / 4 / 5 (4: one VGPR spilled, 5: three)
#endif
constexpr int PM_N = ZT_PM_N;  // start phases decoded side by side per lane

// one start phase's decode: >= 32 valid bits in bb at every step
struct PhaseDec {
  uint64_t bb;
  uint32_t bc, q, rel, ph;
  bool act;
};

// map[x], x = 0 .. maxlen - 1: the phase past s_next at which the decode from
// s_l + x crosses into the next lane (15: it ends the block, breaks, or
// crosses 15 or more bits past it).  ph0 <= 15: map[0] is known (a first
// pass decoded from s_l); 16: decoded here too.  The
// other phases go PM_N at a time: each step issues every decode's next input
// word and primary-table entry before any is used (one LDS round trip per
// step for all of them, where one decode at a time waited for each); a
// literal from the primary table -- nearly every token of these blocks -- is
// consumed inline, anything else takes lane_token.
__device__ uint64_t lane_phase_map(const LaneBits &lb, uint64_t b0, uint32_t s_l, uint32_t limit, bool in_range,
                                   uint32_t ph0, const HuffTab *lt, const HuffTab *dt) {
  constexpr uint32_t M = (1u << PRI) - 1;
  const uint32_t s_next = s_l + SP_LANE_BITS;
  // a token boundary lies within the longest code past s_l when the token
  // straddling s_l is a literal (matches are rare in these blocks; a phase
  // not mapped stays 15 = unknown, and that lane takes the ordinary repair)
  const uint32_t xmax = lt->maxlen < 15 ? (uint32_t)lt->maxlen : 15u;
  uint64_t map = ph0 > 15 ? ~0ull : (~0xFull | ph0);
#pragma unroll 1
  for (uint32_t x0 = ph0 > 15 ? 0u : 1u; x0 < xmax; x0 += PM_N) {
    PhaseDec d[PM_N];
#pragma unroll
    for (int k = 0; k < PM_N; ++k) {
      const uint64_t abs_bit = b0 + s_l + x0 + k;
      const uint32_t q = (uint32_t)(abs_bit >> 5), sh = (uint32_t)abs_bit & 31;
      d[k].bb = (((uint64_t)lb.word(q + 1) << 32) | lb.word(q)) >> sh;
      d[k].bc = 64 - sh;
      d[k].q = q + 2;
      d[k].rel = s_l + x0 + k;
      d[k].ph = 15;
      d[k].act = in_range && x0 + k < xmax;
    }
    for (;;) {  // (per lane: a lane whose phases are all mapped leaves exec; C2 tokenize 5.15 -> 5.03 ms, r05ak)
      bool any = false;
#pragma unroll
      for (int k = 0; k < PM_N; ++k) any = any || d[k].act;
      if (!any) break;
      uint32_t w[PM_N], e[PM_N];
#pragma unroll
      for (int k = 0; k < PM_N; ++k) {
        w[k] = lb.word(d[k].q);
        e[k] = lt->pri[(uint32_t)d[k].bb & M];
      }
#pragma unroll
      for (int k = 0; k < PM_N; ++k) {
        PhaseDec &r = d[k];
        if (!r.act) continue;
        if ((e[k] & 15) && ((e[k] >> 8) & 511) < 256) {
          const uint32_t cl = e[k] & 15;
          r.bb >>= cl;
          r.bc -= cl;
          r.rel += cl;
          if (r.bc <= 32) {
            r.bb |= (uint64_t)w[k] << r.bc;
            r.bc += 32;
            ++r.q;
          }
        } else {
          LaneBits t = lb;
          t.q = r.q;
          t.nw = w[k];  // = word(r.q)
          t.bb = r.bb;
          t.bc = r.bc;
          t.rel = r.rel;
          uint32_t tk, nb;
          const int rr = lane_token(t, lt, dt, tk, nb);
          t.refill();
          r.q = t.q;
          r.bb = t.bb;
          r.bc = t.bc;
          r.rel = t.rel;
          if (rr != 0) {
            r.act = false;
            continue;
          }
        }
        if (r.rel > limit) {
          r.act = false;
        } else if (r.rel >= s_next) {
          const uint32_t dd = r.rel - s_next;
          r.ph = dd < 15 ? dd : 15;
          r.act = false;
        }
      }
    }
#pragma unroll
    for (int k = 0; k < PM_N; ++k)
      if (x0 + k < xmax) map = (map & ~(0xFull << (4 * (x0 + k)))) | ((uint64_t)d[k].ph << (4 * (x0 + k)));
  }
  return map;
}

// (a o b)[x] = a[b[x]] for 16-entry nibble maps
__device__ __forceinline__ uint64_t compose_maps(uint64_t a, uint64_t b) {
  uint64_t r = 0;
#pragma unroll
  for (int x = 0; x < 16; ++x) {
    const uint32_t v = (uint32_t)(b >> (4 * x)) & 15u;
    r |= ((a >> (4 * v)) & 15ull) << (4 * x);
  }
  return r;
}
#endif

// Decode the body of a Huffman block that starts at bit `b0` (relative to
// rd's abase) with the tables in lt / dt.  Tokens go to to.tok[to.ntok ...].
// Returns 0 with *end_bit = the bit after the end-of-block code, 1 when the
// body is too large for this path, or a status.
// stop_rel (bits from b0): decoding also ends at the first token that starts
// at or after it (*stopped = true, *end_bit = that token's start, the token
// not decoded).  bm_out (global, SP_WORDS * 64 words): the token-start bitmap
// of the path's first round (bit x = a token starts at b0 + x), for the
// speculative tokenizer's sync test.
// PHASE: phase maps for near-fixed-length codes (the sync-point / batch
// tokenizer; the general tokenizer keeps them off: their registers cost it a
// wave per SIMD, 3 -> 2, and its units start mid-block anyway)
#ifdef ZT_TK_TIME
// debug: SIMT body decode cycles (lane 0 of each wave): [0] staging, [1] pass 1,
// [2] repairs (phase maps included), [3] pass 2, [4] rounds, [5] repair iterations,
// [6] phase maps + their scan, [7] of [0]: waiting for the previous round's stores
__device__ unsigned long long g_tk_time[8];
#define TK_T(v) v = __builtin_readcyclecounter()
#else
#define TK_T(v) (void)0
#endif
template <bool PHASE = false>
__device__ int tok_huffman_simt(Reader &rd, uint64_t b0, const HuffTab *lt, const HuffTab *dt, TokOut &to,
                                uint64_t &op, SpecShared *sp, uint64_t &end_bit, uint32_t *dump = nullptr,
                                uint32_t stop_rel = 0xFFFFFFFFu, uint32_t *bm_out = nullptr,
                                bool *stopped = nullptr) {
  const int lane = to.lane;
  // bits available after b0 (positions are u32: a body past 2^31 bits -- a
  // 256 MiB single block -- runs into the limit and is reported as broken,
  // which sends the stream to the one-wave decoder)
  const uint64_t lim = uni64(rd.hi) * 8 - b0;
  const uint32_t limit = lim < 0x7FFFFFFFull ? (uint32_t)lim : 0x7FFFFFFFu;
  uint32_t *stage = rd.inbuf;  // the reader's ring is reloaded afterwards
  LaneBits lb;
  lb.stage = stage;
  uint32_t R = 0;  // true start of this round (bits from b0)
  int dump_round = 0;
#ifndef ZT_NO_PHASE_MAPS
  const bool fixedish = PHASE && near_fixed_code(lt);
#endif
  for (;;) {
    [[maybe_unused]] unsigned long long tt0 = 0, tt1 = 0, tt2 = 0, tt3 = 0, tt4 = 0;
    [[maybe_unused]] int n_iter = 0;
    [[maybe_unused]] unsigned long long tph = 0;
#ifndef ZT_NO_PHASE_MAPS
    uint64_t pmap = 0;  // fixedish: this round's phase map of the lane
#endif
    TK_T(tt0);
#ifdef ZT_TK_TIME
    // (measurement: the previous round's token stores, which the stage's
    // loads wait for -- one vmcnt on gfx9)
    unsigned long long ttw;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    TK_T(ttw);
#endif
    // ---- stage the round's input: bytes [a0, a0 + SP_STAGE_BYTES)
    const uint64_t a0 = ((b0 + R) >> 3) & ~uint64_t(15);
    {
      typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
      typedef __attribute__((address_space(1))) const u32x4 g_u32x4;
      const uint64_t hi = uni64(rd.hi);
#pragma unroll
      for (uint32_t k = 0; k < SP_STAGE_BYTES / 1024; ++k) {
        const uint64_t off = a0 + k * 1024 + (uint32_t)lane * 16;
        u32x4 v = {0, 0, 0, 0};
        if (off < hi) v = *(g_u32x4 *)(rd.abase + off);
        const uint32_t w = k * 256 + (uint32_t)lane * 4;
        stage[w] = v.x;
        stage[w + 1] = v.y;
        stage[w + 2] = v.z;
        stage[w + 3] = v.w;
      }
      lb.qbase = (uint32_t)(a0 >> 2);
    }
    for (uint32_t w = 0; w < SP_WORDS; ++w) sp->bm[w][lane] = 0;
    wave_sync();
    TK_T(tt1);
    // ---- pass 1: lane l from s_l past s_{l+1}, marking token starts
    const uint32_t s_l = R + (uint32_t)lane * SP_LANE_BITS;
    const uint32_t s_next = s_l + SP_LANE_BITS;
    const bool in_range = s_l < limit;
    uint32_t end = s_l, ev_pos = 0;  // ev_pos: start of the EOB / invalid token
    int flags = 0;                   // 1 end of block, 2 invalid, 3 stop position reached
    bool todo = in_range;
    uint32_t from = s_l;             // where this lane's current decode starts
    bool repair = false;
#ifndef ZT_NO_PHASE_MAPS
    if (PHASE && fixedish) {
      // near-fixed-length codes: every lane's true start from the composed
      // phase maps at once, instead of a speculative first pass that does not
      // resynchronise on them; the first decode below is then each lane's
      // true path (lanes whose start is unknown wait, as in the repairs)
#ifdef ZT_TK_TIME
      unsigned long long tp0;
      TK_T(tp0);
#endif
      pmap = lane_phase_map(lb, b0, s_l, limit, in_range, 16u, lt, dt);
      uint64_t P = pmap;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const uint32_t lo = (uint32_t)__shfl_up((int)(uint32_t)P, d, 64);
        const uint32_t hi = (uint32_t)__shfl_up((int)(uint32_t)(P >> 32), d, 64);
        const uint64_t q = ((uint64_t)hi << 32) | lo;
        if (lane >= d) P = compose_maps(P, q);
      }
      const uint32_t ph = lane == 0 ? 0u : ((uint32_t)__shfl_up((int)(uint32_t)P, 1, 64) & 15u);
      todo = in_range && ph < 15;
      from = s_l + ph;
      repair = true;  // (the bitmap is empty: nothing to merge with)
#ifdef ZT_TK_TIME
      unsigned long long tp1;
      TK_T(tp1);
      tph += tp1 - tp0;
#endif
    }
#endif
    for (int iter = 0;; ++iter) {
      if (iter > 66) return ZT_E_INPUT_BROKEN;
      bool active = todo;
      uint32_t cw = 0, cwi = 0;  // bitmap word being assembled, its index
      if (active) {
        lb.init(b0 + from, from);
        cwi = (from - s_l) >> 5;
        cw = 0;
        if (!repair) flags = 0;
        // marks below a repair's start are off every path it can merge with
        for (uint32_t x = 0; x < cwi; ++x) sp->bm[x][lane] = 0;
      }
      // (a per-lane loop: finished lanes leave exec with their registers
      // untouched, where a wave loop around `if (active)` copied the carried
      // state every iteration -- tokenize 3.86 -> 3.60 ms per GiB, r05ai)
      while (active) {
        const uint32_t p = lb.rel - s_l;  // < SP_LANE_BITS while decoding this lane's range
        const uint32_t wi = p >> 5;
        if (wi != cwi) {
          // leave word cwi: new marks below, on a repair old marks are stale
          sp->bm[cwi][lane] = cw;
          for (uint32_t x = cwi + 1; x < wi; ++x) sp->bm[x][lane] = 0;
          cwi = wi;
          cw = 0;
        }
        if (repair && ((sp->bm[wi][lane] >> (p & 31)) & 1)) {
          // merged with the old path: the old marks from p on are right
          const uint32_t below = (p & 31) ? (0xFFFFFFFFu >> (32 - (p & 31))) : 0u;
          sp->bm[wi][lane] = (cw & below) | (sp->bm[wi][lane] & ~below);
          active = false;
        } else {
          cw |= 1u << (p & 31);
          if (lb.rel >= stop_rel) {
            // a token starts at or after the stop: the unit ends here
            flags = 3;
            ev_pos = s_l + p;
            end = ev_pos;
            active = false;
          } else {
            const int r = lane_skip(lb, lt, dt);
            if (r != 0 || lb.rel > limit) {
              flags = r > 0 ? 1 : 2;
              ev_pos = s_l + p;
              end = lb.rel;
              active = false;
            } else if (lb.rel >= s_next) {
              end = lb.rel;
              flags = 0;
              active = false;
            }
          }
          if (!active) {
            sp->bm[cwi][lane] = cw;
            for (uint32_t x = cwi + 1; x < SP_WORDS; ++x) sp->bm[x][lane] = 0;
          }
        }
      }
      wave_sync();
#ifdef ZT_TK_TIME
      if (iter == 0) TK_T(tt2);
      n_iter = iter;
#endif
      // ---- which lanes are on the true path?
      const uint32_t t = from_prev_lane(end, R);
      const uint32_t tp = t - s_l;
      const bool synced = in_range && t >= s_l && tp < SP_LANE_BITS && ((sp->bm[tp >> 5][lane] >> (tp & 31)) & 1);
      const uint64_t U = __ballot(!synced);
      const uint64_t E = __ballot(synced && flags != 0 && ev_pos >= t);
      const int f = U ? __builtin_ctzll(U) : 64;
      const int e = E ? __builtin_ctzll(E) : 64;
      if (e < f) {
        // the block ends (or breaks) in lane e
        if (__builtin_amdgcn_readlane(flags, e) == 2) return ZT_E_INVALID_SYMBOL;
        break;
      }
      if (f == 64) break;  // every lane synchronised, the block continues
      if (!__builtin_amdgcn_readlane((int)in_range, f)) return ZT_E_INPUT_BROKEN;  // runs past the input
#ifndef ZT_NO_PHASE_MAPS
      // Phase maps: lanes below f are on the true path and lane f's true
      // start t_f is exact; every later lane's start comes from the maps
      // composed from t_f's phase (lane f - 1's map replaced by that
      // constant).  A lane whose start is unknown (a token 15 or more bits
      // past a lane start, or a path that ends or breaks before it) waits:
      // once the lanes before it are repaired it becomes lane f, and the maps
      // carry on from there -- one iteration per such lane, where the
      // ordinary repairs fixed one lane per iteration from it on.
      if (PHASE && fixedish && f > 0) {
        const uint32_t tf = __builtin_amdgcn_readlane(t, f);
        const uint32_t sf = R + (uint32_t)f * SP_LANE_BITS;
        const uint32_t phf = (tf >= sf && tf - sf < 15) ? tf - sf : 15u;
        uint64_t P = lane == f - 1 ? 0x1111111111111111ull * phf : pmap;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
          const uint32_t lo = (uint32_t)__shfl_up((int)(uint32_t)P, d, 64);
          const uint32_t hi = (uint32_t)__shfl_up((int)(uint32_t)(P >> 32), d, 64);
          const uint64_t q = ((uint64_t)hi << 32) | lo;
          if (lane >= d) P = compose_maps(P, q);
        }
        const uint32_t ph = (uint32_t)__shfl_up((int)(uint32_t)P, 1, 64) & 15u;  // (map_{l-1} o ... o map_0)[0]
        if (lane < f) {
          todo = false;
        } else if (lane == f) {
          todo = in_range && t >= s_l && tp < SP_LANE_BITS;
          from = t;
        } else {
          const bool known = in_range && ph < 15;
          const bool marked = known && ((sp->bm[ph >> 5][lane] >> (ph & 31)) & 1);
          todo = known && !marked;
          from = s_l + ph;
        }
        repair = true;
        continue;
      }
#endif
      // re-decode every unsynchronised lane from its (current) true start
      // (a lane whose predecessor stopped short of it waits: that predecessor
      // is off the true path and is repaired first)
      todo = in_range && !synced && t >= s_l && tp < SP_LANE_BITS;
      if (todo) from = t;
      repair = true;
    }
    TK_T(tt3);
    // final per-lane state: true start t, tokens = marks in [t, ev or end)
    const uint32_t t = from_prev_lane(end, R);
    const uint64_t E = __ballot(flags != 0 && ev_pos >= t && in_range);
    const int e = E ? __builtin_ctzll(E) : 64;
    const int last = e < 64 ? e : 63;
    const bool eob = e < 64;
    const bool use = lane <= last;
    uint32_t my_tok = 0;
    if (use) {
      const uint32_t lo = t - s_l;
      const uint32_t hi_p = (lane == e) ? ev_pos - s_l : SP_LANE_BITS;  // marks at p < hi_p
      for (uint32_t w = lo >> 5; w < SP_WORDS && w * 32 < hi_p; ++w) {
        uint32_t m = sp->bm[w][lane];
        if (w == (lo >> 5)) m &= 0xFFFFFFFFu << (lo & 31);
        if (hi_p < (w + 1) * 32) m &= (hi_p & 31) ? (0xFFFFFFFFu >> (32 - (hi_p & 31))) : 0u;
        my_tok += __popc(m);
      }
    }
    if (bm_out && R == 0) {
      // the path's token starts of this first round: lane l's marks in [t, hi_p)
      const uint32_t lo = t - s_l;
      const uint32_t hi_p = (lane == e) ? ev_pos - s_l : SP_LANE_BITS;
      for (uint32_t w = 0; w < SP_WORDS; ++w) {
        uint32_t m = use ? sp->bm[w][lane] : 0u;
        if (w * 32 + 32 <= lo) m = 0;
        else if (w * 32 < lo) m &= 0xFFFFFFFFu << (lo & 31);
        if (hi_p <= w * 32) m = 0;
        else if (hi_p < (w + 1) * 32) m &= 0xFFFFFFFFu >> (32 - (hi_p & 31));
        bm_out[lane * SP_WORDS + w] = m;
      }
    }
    if (dump && dump_round < 8) {
      uint32_t *d = dump + (dump_round * 64 + lane) * 8;
      d[0] = R;
      d[1] = t;
      d[2] = end;
      d[3] = my_tok;
      d[4] = (uint32_t)e;
      d[5] = (uint32_t)flags;
      d[6] = (uint32_t)last;
      d[7] = ev_pos;
      ++dump_round;
    }
    uint32_t tok_incl = my_tok;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const uint32_t a = __shfl_up(tok_incl, off, 64);
      if (lane >= off) tok_incl += a;
    }
    const uint32_t tot_tok = __builtin_amdgcn_readlane(tok_incl, last);
    const uint32_t nt0 = uni(to.ntok);
    if ((uint64_t)nt0 + tot_tok > to.cap) return ZT_E_NOMEM;
    const uint32_t r_end = eob ? __builtin_amdgcn_readlane(end, e) : __builtin_amdgcn_readlane(end, 63);
    // ---- pass 2: exact ranges, tokens written at their index
    const uint32_t nt1 = nt0 + tot_tok;
    const uint32_t tail_base = nt1 & ~63u;
    to.flush_partial();
    sp->tail[lane] = to.stg;
    wave_sync();
    uint32_t idx = nt0 + tok_incl - my_tok;
    const uint32_t idx_end = idx + my_tok;
    uint32_t my_by = 0;
    bool active = use && my_tok > 0;
    uint32_t *tokp = to.tok;
#ifndef ZT_TK_SEQ_PASS2
    // every token start of the lane's exact range [t, hi_p) is marked, so the
    // tokens are decoded independently of each other (no bit position carried
    // from one to the next), up to 4 at a time: one aligned group of 4 token
    // indices per step, stored as one 16-byte store when the lane fills it
    const bool vec_ok = (reinterpret_cast<uintptr_t>(tokp) & 15) == 0;
    uint32_t mw = 0, mm = 0;  // mark word index and its unvisited marks
    if (active) {
      const uint32_t lo = t - s_l;
      mw = lo >> 5;
      mm = sp->bm[mw][lane] & (0xFFFFFFFFu << (lo & 31));
    }
    while (__ballot(active)) {
      if (active) {
        const uint32_t nk0 = 4 - (idx & 3), left = idx_end - idx;
        const uint32_t nk = nk0 < left ? nk0 : left;
        uint32_t xs[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          xs[k] = 0;
          if ((uint32_t)k < nk) {
            while (mm == 0 && mw + 1 < SP_WORDS) mm = sp->bm[++mw][lane];  // (bounded: a count mismatch cannot spin)
            xs[k] = s_l + mw * 32 + (uint32_t)__builtin_ctz(mm);
            mm &= mm - 1;
          }
        }
        uint32_t tk[4], nb[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          tk[k] = 0;
          nb[k] = 0;
          if ((uint32_t)k < nk) token_at(stage, lb.qbase, b0 + xs[k], lt, dt, tk[k], nb[k]);
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          my_by += nb[k];
          if ((uint32_t)k < nk && idx + k >= tail_base) sp->tail[(idx + k) & 63] = tk[k];
        }
        if (vec_ok && nk == 4) {
          typedef unsigned int u32x4s __attribute__((ext_vector_type(4)));
          *reinterpret_cast<u32x4s *>(tokp + idx) = u32x4s{tk[0], tk[1], tk[2], tk[3]};
        } else {
#pragma unroll
          for (int k = 0; k < 4; ++k)
            if ((uint32_t)k < nk) tokp[idx + k] = tk[k];
        }
        idx += nk;
        if (idx >= idx_end) active = false;
      }
    }
#else
    if (active) lb.init(b0 + t, t);
    while (__ballot(active)) {
      if (active) {
        uint32_t tk = 0, nb = 0;
        lane_token(lb, lt, dt, tk, nb);
        tokp[idx] = tk;
        my_by += nb;
        if (idx >= tail_base) sp->tail[idx & 63] = tk;
        if (++idx >= idx_end) active = false;
      }
    }
#endif
    wave_sync();
    uint32_t by = my_by;
#pragma unroll
    for (int off = 32; off; off >>= 1) by += __shfl_xor(by, off, 64);
    to.ntok = nt1;
    to.stg = sp->tail[lane];
    op += uni(by);
#ifdef ZT_TK_TIME
    TK_T(tt4);
    if (lane == 0) {
      atomicAdd(&g_tk_time[0], tt1 - tt0);
      atomicAdd(&g_tk_time[1], tt2 - tt1);
      atomicAdd(&g_tk_time[2], tt3 - tt2);
      atomicAdd(&g_tk_time[3], tt4 - tt3);
      atomicAdd(&g_tk_time[4], 1ull);
      atomicAdd(&g_tk_time[5], (unsigned long long)n_iter);
      atomicAdd(&g_tk_time[6], tph);
      atomicAdd(&g_tk_time[7], ttw - tt0);
    }
#endif
    if (eob) {
      end_bit = b0 + r_end;
      if (stopped) *stopped = __builtin_amdgcn_readlane(flags, e) == 3;
      return ZT_OK;
    }
    R = r_end;
  }
}

// ---- token -> byte resolution constants (inflate_tok.hip, inflate_gen.hip)
__device__ __forceinline__ uint32_t bperm(uint32_t v, uint32_t src_lane) {
  return (uint32_t)__builtin_amdgcn_ds_bpermute((int)(src_lane << 2), (int)v);
}
#ifndef ZT_RS_TOK_RING
#define ZT_RS_TOK_RING 512  // 3.3 KiB of expand LDS: 8 waves per SIMD (1024: 29 waves per CU; expand 2.75 -> 2.51 ms per GiB)
#endif
#ifndef ZT_RS_AHEAD
#define ZT_RS_AHEAD 6
#endif
constexpr uint32_t RS_TOK_RING = ZT_RS_TOK_RING;  // expand: tokens staged in LDS (chunks of 64)
constexpr uint32_t RS_AHEAD = ZT_RS_AHEAD;        // chunks in flight ahead of the cursor
static_assert((RS_AHEAD + 2) * 64 <= RS_TOK_RING, "expand token ring");
constexpr uint32_t RS_FLUSH = 8192;           // output flush granule
#ifndef ZT_CP_STEP
#define ZT_CP_STEP 1024  // 512: copy_kernel 1.063 ms, expand 2.063 ms per GiB; 1024: 0.840 / 2.088 (profiles/r04cp_*)
#endif
constexpr uint32_t CP_STEP = ZT_CP_STEP;  // copy_kernel bytes per step (a multiple of 256)
constexpr int CP_G = CP_STEP / 256;       // 4-byte groups per lane per step
#ifndef ZT_CP_RING
#define ZT_CP_RING 4096
#endif
#ifndef ZT_CP_AHEAD
#define ZT_CP_AHEAD 6
#endif
constexpr uint32_t CP_CHUNK = 512;              // descriptors per LDS-DMA instruction (16 bytes per lane)
constexpr uint32_t CP_DESC_RING = ZT_CP_RING;  // descriptors staged in LDS
constexpr uint32_t CP_AHEAD = ZT_CP_AHEAD;      // chunks in flight ahead of the step's
static_assert(CP_STEP % 256 == 0 && (CP_STEP & (CP_STEP - 1)) == 0, "copy step");
static_assert((CP_AHEAD + (CP_STEP + CP_CHUNK - 1) / CP_CHUNK) * CP_CHUNK <= CP_DESC_RING && CP_AHEAD < 64,
              "descriptor ring");
// s_waitcnt vmcnt(v) with lgkmcnt / expcnt left alone (vmcnt bits 3:0 and 15:14)
constexpr int cp_vmcnt(uint32_t v) { return (int)(0x0F70u | (v & 15u) | ((v >> 4) << 14)); }

// copy kernels: descriptor chunks up to CP_AHEAD past the ones step [op, op +
// CP_STEP) reads are in flight (one 1 KiB LDS-DMA each, dsrc 1 KiB aligned,
// its buffer padded by a chunk), and the step's own have landed
typedef unsigned int cp_u32x4 __attribute__((ext_vector_type(4)));
// (U: the offset type -- uint32_t for segments below 2^31 bytes, where every
// index here stays below 2^32 and the bookkeeping is 32-bit scalar work)
template <typename U = uint64_t>
__device__ __forceinline__ void cp_desc_fetch(const uint16_t *dsrc, uint16_t *ring, U op, U n, U &issued, int lane) {
  const U nchunks = (n + CP_CHUNK - 1) / CP_CHUNK;
  const U need0 = (op + CP_STEP + CP_CHUNK - 1) / CP_CHUNK;
  const U need = need0 < nchunks ? need0 : nchunks;
  const U want = need + CP_AHEAD < nchunks ? need + CP_AHEAD : nchunks;
  while (issued < want) {
    __builtin_amdgcn_global_load_lds(reinterpret_cast<const cp_u32x4 *>(dsrc + issued * CP_CHUNK) + lane,
                                     ring + ((issued * CP_CHUNK) & (CP_DESC_RING - 1)), 16, 0, 0);
    ++issued;
  }
  if (issued - need >= CP_AHEAD)
    __builtin_amdgcn_s_waitcnt(cp_vmcnt(CP_AHEAD));
  else
    __builtin_amdgcn_s_waitcnt(0x0F70);
}

}  // namespace
}  // namespace zt
