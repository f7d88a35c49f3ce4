// inflate_tok.hip -- two-phase inflate of streams that carry block sync points.
//
// Huffman decoding never needs history; LZ77 resolution needs only output
// bytes.  The decode is therefore split where the dependency structure
// splits (replaces src/RawInflate.ts:127-143 / :466-516 for such streams):
//
//   A. tokenize_kernel -- one wavefront per *unit*: a unit starts at a byte
//      aligned block start (a sync point: the byte after an empty stored
//      block, 00 00 FF FF, which this engine's deflate writes after every
//      32 KiB block) and decodes blocks until the next block start is again a
//      sync point.  It needs only its decode tables in LDS (no history ring),
//      so many units run per CU.  Output: one u32 token per literal
//      (the byte) or match (length << 16 | distance); stored bytes become
//      literal tokens.  Units that start at a false sync point (the pattern
//      inside data) decode garbage and are simply not on the chain.
//   B. resolve_kernel -- one wavefront per *segment* (restart points: the
//      10-byte double marker; no match reaches behind one): 64 output bytes
//      per step, byte-parallel.  Each lane finds its token with a start-mark
//      ballot, takes a literal or reads the 32 KiB LDS history ring, and
//      in-window back references (overlapping copies) are resolved by pointer
//      jumping over the window (<= 6 bpermute rounds).  Output goes straight
//      to its final offset in HBM.
// The host follows the chain of units from the stream start, so only units
// that are really on the stream's block sequence are used; any error on the
// chain (or a match reaching behind a segment start) returns to the caller,
// which decodes the stream with one wave and reports the exact error.
#include "inflate_common.h"

namespace zt {

namespace {


struct TokShared {
  uint32_t inbuf[IN_RING_WORDS + 4];
  HuffTab lit;
  HuffTab dist;
  uint8_t lens[320];
};

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
#define ZT_SP_LANE_BITS 480
#endif
constexpr uint32_t SP_LANE_BITS = ZT_SP_LANE_BITS;        // 60 bytes per lane: 18.5 KiB of LDS, 8 units per CU
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
    bb = word(q) >> sh;
    bc = 32 - sh;
    ++q;
    rel = rel0;
  }
  // afterwards at least 32 valid bits
  __device__ __forceinline__ void refill() {
    if (bc <= 32) {
      bb |= (uint64_t)word(q) << bc;
      bc += 32;
      ++q;
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

// lane l-1's value (lane 0: `first`), with every lane taking part (DPP wave_shr:1)
__device__ __forceinline__ uint32_t from_prev_lane(uint32_t v, uint32_t first) {
  return (uint32_t)__builtin_amdgcn_update_dpp((int)first, (int)v, 0x138, 0xF, 0xF, false);
}

// Decode the body of a Huffman block that starts at bit `b0` (relative to
// rd's abase) with the tables in lt / dt.  Tokens go to to.tok[to.ntok ...].
// Returns 0 with *end_bit = the bit after the end-of-block code, 1 when the
// body is too large for this path, or a status.
__device__ int tok_huffman_simt(Reader &rd, uint64_t b0, const HuffTab *lt, const HuffTab *dt, TokOut &to,
                                uint64_t &op, SpecShared *sp, uint64_t &end_bit, uint32_t *dump = nullptr) {
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
  for (;;) {
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
    // ---- pass 1: lane l from s_l past s_{l+1}, marking token starts
    const uint32_t s_l = R + (uint32_t)lane * SP_LANE_BITS;
    const uint32_t s_next = s_l + SP_LANE_BITS;
    const bool in_range = s_l < limit;
    uint32_t end = s_l, ev_pos = 0;  // ev_pos: start of the EOB / invalid token
    int flags = 0;                   // 1 end of block, 2 invalid
    bool todo = in_range;
    uint32_t from = s_l;             // where this lane's current decode starts
    bool repair = false;
    for (int iter = 0;; ++iter) {
      if (iter > 66) return ZT_E_INPUT_BROKEN;
      bool active = todo;
      uint32_t cw = 0, cwi = 0;  // bitmap word being assembled, its index
      uint32_t merge = 0xFFFFFFFFu;
      if (active) {
        lb.init(b0 + from, from);
        cwi = (from - s_l) >> 5;
        cw = 0;
        if (!repair) flags = 0;
        // marks below a repair's start are off every path it can merge with
        for (uint32_t x = 0; x < cwi; ++x) sp->bm[x][lane] = 0;
      }
      while (__ballot(active)) {
        if (active) {
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
            merge = p;
            const uint32_t below = (p & 31) ? (0xFFFFFFFFu >> (32 - (p & 31))) : 0u;
            sp->bm[wi][lane] = (cw & below) | (sp->bm[wi][lane] & ~below);
            active = false;
          } else {
            cw |= 1u << (p & 31);
            uint32_t tk, nb;
            const int r = lane_token(lb, lt, dt, tk, nb);
            if (r != 0 || lb.rel > limit) {
              flags = r > 0 ? 1 : 2;
              ev_pos = lb.rel - 0;  // provisional; fixed below
              ev_pos = s_l + p;
              end = lb.rel;
              active = false;
            } else if (lb.rel >= s_next) {
              end = lb.rel;
              flags = 0;
              active = false;
            }
            if (!active) {
              sp->bm[cwi][lane] = cw;
              for (uint32_t x = cwi + 1; x < SP_WORDS; ++x) sp->bm[x][lane] = 0;
            }
          }
        }
      }
      wave_sync();
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
      // re-decode every unsynchronised lane from its (current) true start
      // (a lane whose predecessor stopped short of it waits: that predecessor
      // is off the true path and is repaired first)
      todo = in_range && !synced && t >= s_l && tp < SP_LANE_BITS;
      if (todo) from = t;
      repair = true;
      (void)merge;
    }
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
    if (active) lb.init(b0 + t, t);
    uint32_t *tokp = to.tok;
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
    wave_sync();
    uint32_t by = my_by;
#pragma unroll
    for (int off = 32; off; off >>= 1) by += __shfl_xor(by, off, 64);
    to.ntok = nt1;
    to.stg = sp->tail[lane];
    op += uni(by);
    if (eob) {
      end_bit = b0 + r_end;
      return ZT_OK;
    }
    R = r_end;
  }
}

__global__ __launch_bounds__(64) void tokenize_kernel(TokParams P) {
  __shared__ TokShared sh;
  __shared__ SpecShared spsh;
  const uint32_t u = blockIdx.x;
  const int lane = threadIdx.x & 63;
  const TokJob job = P.jobs[u];
  const uint64_t n = job.end ? job.end : P.n;
  Reader rd;
  rd.init(P.in, n, job.start, sh.inbuf, lane);
  TokOut to;
  to.tok = P.tokens + job.tok_off;
  to.cap = job.tok_cap;
  to.ntok = 0;
  to.stg = 0;
  to.lane = lane;
  uint64_t op = 0;
  int status = ZT_OK, detail = 0, stop_idx = -1;
  uint64_t si = job.stop_first;
  bool bfinal = false;
  g_u8 *gin = (g_u8 *)P.in;
  while (!bfinal) {
    uint32_t v;
    if (!rd.template bits<false>(3, v)) {
      status = ZT_E_INPUT_BROKEN;
      break;
    }
    bfinal = v & 1;
    const uint32_t btype = v >> 1;
    if (btype == 0) {
      // stored block (src/RawInflate.ts:251-318): bytes become literal tokens
      uint64_t p = (rd.pos_bits_in() + 7) >> 3;
      if (p + 4 > n) {
        status = ZT_E_STORED_LEN;
        break;
      }
      const uint32_t len = (uint32_t)gin[p] | ((uint32_t)gin[p + 1] << 8);
      p += 4;
      if (p + len > n) {
        status = ZT_E_INPUT_BROKEN;
        break;
      }
      const uint32_t nt0 = uni(to.ntok);
      if (nt0 + len > to.cap) {
        status = ZT_E_NOMEM;
        break;
      }
      if (len) {
        to.flush_partial();
        for (uint32_t j = lane; j < len; j += 64) to.tok[nt0 + j] = gin[p + j];
        const uint32_t nt = nt0 + len;
        const uint32_t idx = (nt & ~63u) + (uint32_t)lane;
        if ((uint32_t)lane < (nt & 63) && idx >= nt0) to.stg = gin[p + idx - nt0];
        to.ntok = nt;
        op += len;
      }
      rd.seek_byte(p + len);
    } else {
      status = read_tables<false>(rd, sh.lens, &sh.lit, &sh.dist, btype, lane, detail);
      if (status) break;
      uint64_t end_bit = 0;
      const uint64_t body0 = rd.pos_bits();
      const uint32_t nt_before = uni(to.ntok);
      const uint64_t op_before = op;
      uint32_t *dump = (P.dbg && u == P.dump_unit && P.dump_once == 0) ? reinterpret_cast<uint32_t *>(P.dbg + (uint64_t)P.count * 8) : nullptr;
      int r = P.simt ? tok_huffman_simt(rd, body0, &sh.lit, &sh.dist, to, op, &spsh, end_bit, dump) : 1;
      if (P.dbg && r == 0) {
        // shadow check: decode the same body with one lane and compare
        const uint64_t s_end = end_bit, s_op = op;
        const uint32_t s_nt = uni(to.ntok);
        rd.seek_bit(body0);
        to.ntok = nt_before;
        to.stg = 0;
        op = op_before;
        r = tok_huffman(rd, &sh.lit, &sh.dist, to, op);
        const uint64_t c_end = rd.pos_bits();
        if (lane == 0 && (c_end != s_end || uni(to.ntok) != s_nt || op != s_op)) {
          uint64_t *d = P.dbg + (uint64_t)u * 8;
          if (d[0] == 0) {
            d[0] = 1;
            d[1] = body0;
            d[2] = s_end;
            d[3] = c_end;
            d[4] = s_nt - nt_before;
            d[5] = uni(to.ntok) - nt_before;
            d[6] = s_op - op_before;
            d[7] = op - op_before;
          }
        }
        if (r == 0) r = 2;  // already decoded (position is current)
      }
      if (r == 2) {
        r = 0;
      } else if (r == 1) {
        status = tok_huffman(rd, &sh.lit, &sh.dist, to, op);
      } else if (r == 0) {
        rd.seek_bit(end_bit);
      } else {
        status = r;
      }
      if (status) break;
    }
    if (!bfinal) {
      // the unit ends where the next block starts on a sync point
      const uint64_t pb = rd.pos_bits_in();
      if ((pb & 7) == 0) {
        const uint64_t q = pb >> 3;
        while (si < P.nstops && P.stops[si] < q) ++si;
        if (si < P.nstops && P.stops[si] == q) {
          stop_idx = (int)si;
          break;
        }
      }
    }
  }
  to.flush_partial();
  if (lane == 0) {
    TokResult r;
    r.out_len = op;
    r.end_bits = rd.pos_bits_in();
    r.ntok = to.ntok;
    r.status = status;
    r.detail = detail;
    r.stop_idx = stop_idx;
    P.res[u] = r;
  }
}

// ---------------------------------------------------------------- phase B
__device__ __forceinline__ uint32_t bperm(uint32_t v, uint32_t src_lane) {
  return (uint32_t)__builtin_amdgcn_ds_bpermute((int)(src_lane << 2), (int)v);
}

// inclusive prefix sum over the wave (DPP row shifts + row broadcasts)
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t x) {
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xF, 0xF, true);  // row_shr:1
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xF, 0xF, true);  // row_shr:2
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xF, 0xF, true);  // row_shr:4
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xF, 0xF, true);  // row_shr:8
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xA, 0xF, false); // row_bcast:15
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xC, 0xF, false); // row_bcast:31
  return x;
}

__device__ __forceinline__ uint32_t tok_len(uint32_t t) { return (t >> 16) ? (t >> 16) : 1u; }

constexpr uint32_t RS_TOK_RING = 1024;        // tokens staged in LDS (16 chunks of 64)
constexpr uint32_t RS_AHEAD = 12;             // chunks in flight ahead of the cursor
constexpr uint32_t RS_FLUSH = 8192;           // output flush granule

// Phase B runs in two kernels.
//
// B0 expand_kernel -- one wavefront per unit (many per CU: no history
//   needed): tokens -> one u16 *descriptor* per output byte, written at the
//   byte's final position: 0x8000 | byte for a literal, else D - 1 where the
//   byte equals the output byte D positions back.  For byte k of a match
//   (length L, distance d) the source is taken before the match start,
//   start - d + (k mod d), so D = d * (1 + k / d) <= 32768, and a match never
//   depends on itself.  64 bytes per step: each lane finds its token with a
//   start-mark ballot over the scanned token lengths.
// B1 copy_kernel -- one wavefront per segment, sequential over its bytes,
//   64 per step: a literal, or a read of the 32 KiB LDS history ring; bytes
//   whose source lies inside the step are resolved by pointer jumping.  The
//   output goes through the ring to HBM in 8 KiB granules.
constexpr uint32_t CP_STEP = 256;  // copy_kernel bytes per step

struct ExpandShared {
  uint32_t tok[RS_TOK_RING];   // token chunks, filled by LDS-DMA
  uint32_t mark[64];
  uint16_t cw[CP_STEP];        // descriptors of the current copy step
};

__global__ __launch_bounds__(64) void expand_kernel(ResolveParams P) {
  __shared__ ExpandShared sh;
  const uint32_t u = blockIdx.x;
  const int lane = threadIdx.x & 63;
  const ChainUnit cu = P.units[u];
  const uint32_t *tk = P.tokens + cu.tok_off;
  const uint32_t ntok = cu.ntok;
  const uint32_t nchunks = (ntok + 63) / 64;
  uint16_t *desc = P.desc + cu.desc_off;
  const uint64_t back = cu.out_off - cu.seg_off;  // bytes of the segment before this unit
  sh.mark[lane] = 0;
  uint32_t seq = 0;
  uint32_t issued = 0;
  uint32_t cur = 0, rem = 0;
  uint32_t op = 0;  // unit-relative output position
  bool bad = false;
  while (cur < ntok) {
    const uint32_t need = (cur >> 6) + 2 < nchunks ? (cur >> 6) + 2 : nchunks;
    const uint32_t want = need + RS_AHEAD < nchunks ? need + RS_AHEAD : nchunks;
    while (issued < want) {
      __builtin_amdgcn_global_load_lds(tk + (uint64_t)issued * 64 + lane,
                                       &sh.tok[(issued * 64) & (RS_TOK_RING - 1)], 4, 0, 0);
      ++issued;
    }
    if (issued - need >= RS_AHEAD)
      __builtin_amdgcn_s_waitcnt(0x0F70 | RS_AHEAD);  // vmcnt(RS_AHEAD)
    else
      __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
    const uint32_t ti = cur + (uint32_t)lane;
    const bool valid = ti < ntok;
    const uint32_t t = sh.tok[ti & (RS_TOK_RING - 1)];
    const uint32_t len = valid ? tok_len(t) : 0u;
    const uint32_t S = wave_incl_scan(len);
    const uint32_t total = (uint32_t)__builtin_amdgcn_readlane((int)S, 63) - rem;
    // windows coincide with copy_kernel's 64-byte steps of the segment
    const uint64_t pos = back + op;  // segment position of this window's first byte
    const uint32_t room = 64 - (uint32_t)(pos & 63);
    const uint32_t W = total < room ? total : room;
    const uint64_t ws = pos & ~uint64_t(CP_STEP - 1);
    ++seq;
    const int32_t p = (int32_t)S - (int32_t)rem;
    if (valid && p > 0 && p < 64) sh.mark[p] = seq;
    wave_sync();
    const uint64_t starts = __ballot(sh.mark[lane] == seq);
    const uint32_t owner = __popcll(starts & (~0ull >> (63 - lane)));  // token of byte `lane`
    const uint32_t tj = bperm(t, owner);
    const uint32_t ej = bperm(S - len, owner);  // the token's start, relative to the cursor token
    // descriptor: 0x8000 | byte (literal), 0x8100 | o (= byte ws + o, before
    // this unit), or ws - src - 1 (a byte before the copy step); references
    // into the step are followed here (earlier windows from LDS, this window
    // by pointer jumping over the lanes)
    uint32_t dsc = 0x8000u;
    int32_t ptr = -1;
    if ((uint32_t)lane < W) {
      if ((tj >> 16) == 0) {
        dsc = 0x8000u | (tj & 0xFF);
      } else {
        const uint32_t dist = tj & 0xFFFF;
        const uint32_t k = rem + (uint32_t)lane - ej;  // byte index inside the match
        const uint32_t D = k < dist ? dist : dist * (1 + k / dist);
        const uint64_t x = pos + lane;
        if ((uint64_t)D > x) {
          bad = true;  // reaches behind the segment start
        } else {
          const uint64_t src = x - D;
          if (src < ws)
            dsc = (uint32_t)(ws - src - 1);
          else if (src < back)
            dsc = 0x8100u | (uint32_t)(src - ws);  // before this unit: copy_kernel resolves it
          else if (src < pos)
            dsc = sh.cw[src - ws];  // an earlier window of this step, already resolved
          else
            ptr = (int32_t)(src - pos);
        }
      }
    }
    while (__ballot(ptr >= 0)) {
      const uint32_t q = ptr >= 0 ? (uint32_t)ptr : (uint32_t)lane;
      const uint32_t d2 = bperm(dsc, q);
      const int32_t p2 = (int32_t)bperm((uint32_t)ptr, q);
      if (ptr >= 0) {
        if (p2 < 0) {
          dsc = d2;
          ptr = -1;
        } else {
          ptr = p2;
        }
      }
    }
    if ((uint32_t)lane < W) {
      desc[op + lane] = (uint16_t)dsc;
      sh.cw[pos - ws + lane] = (uint16_t)dsc;
    }
    wave_sync();
    op += W;
    const uint64_t done = __ballot(valid && S <= rem + W);
    const uint32_t kdone = (uint32_t)__popcll(done);
    const uint32_t s_last = kdone ? (uint32_t)__builtin_amdgcn_readlane((int)S, kdone - 1) : 0u;
    rem = rem + W - s_last;
    cur += kdone;
  }
  const bool any_bad = __ballot(bad) != 0;
  if (lane == 0) P.unit_status[u] = any_bad ? ZT_E_INVALID_DISTANCE : (op != cu.out_len ? ZT_E_INPUT_BROKEN : ZT_OK);
}

typedef unsigned int u32x4r __attribute__((ext_vector_type(4)));

#ifndef ZT_CP_RING
#define ZT_CP_RING 2048
#endif
#ifndef ZT_CP_AHEAD
#define ZT_CP_AHEAD 12
#endif
constexpr uint32_t CP_DESC_RING = ZT_CP_RING;  // descriptors staged in LDS (chunks of 128)
constexpr uint32_t CP_AHEAD = ZT_CP_AHEAD;      // chunks in flight ahead of the step
static_assert((CP_AHEAD + 2) * 128 <= CP_DESC_RING && CP_AHEAD < 64, "descriptor ring");
// s_waitcnt vmcnt(v) with lgkmcnt / expcnt left alone (vmcnt bits 3:0 and 15:14)
constexpr int cp_vmcnt(uint32_t v) { return (int)(0x0F70u | (v & 15u) | ((v >> 4) << 14)); }

struct CopyShared {
  uint8_t ring[RING];                        // 32 KiB history, also the output staging
  uint16_t desc[CP_DESC_RING];               // descriptor chunks, filled by LDS-DMA
};

// ring bytes [lo, hi) (segment positions) to out + lo
__device__ __forceinline__ void cp_flush(const CopyShared *sh, uint8_t *out, uint64_t lo, uint64_t hi, int lane) {
  if (lo >= hi) return;
  if ((((uintptr_t)out + lo) & 15) == 0 && ((hi - lo) & 15) == 0) {
    for (uint64_t p = lo + (uint64_t)lane * 16; p < hi; p += 1024)
      *reinterpret_cast<u32x4r *>(out + p) = *reinterpret_cast<const u32x4r *>(&sh->ring[p & RING_MASK]);
  } else {
    for (uint64_t p = lo + lane; p < hi; p += 64) out[p] = sh->ring[p & RING_MASK];
  }
}

// one descriptor -> byte, or -1 for "the byte op + off of this step"
// (branch-free: the ring is read for every descriptor, the literal selected
// after -- per-byte branches cost more issue slots than the extra LDS read)
__device__ __forceinline__ uint32_t cp_byte(const CopyShared *sh, uint64_t op, uint32_t d, int32_t &off) {
  const uint32_t rv = sh->ring[((uint32_t)op - d - 1) & RING_MASK];
  const bool lit = (d & 0x8000u) != 0;
  off = (lit && (d & 0x100u)) ? (int32_t)(d & 0xFF) : -1;
  return lit ? (d & 0xFF) : rv;
}

__global__ __launch_bounds__(64) void copy_kernel(ResolveParams P) {
  __shared__ CopyShared sh;
  const uint32_t sg = blockIdx.x;
  const int lane = threadIdx.x & 63;
  const SegJob sj = P.segs[sg];
  const uint64_t seg_out = P.units[sj.first].out_off;
  const ChainUnit lastu = P.units[sj.first + sj.count - 1];
  const uint64_t n = lastu.out_off + lastu.out_len - seg_out;  // segment bytes
  uint8_t *out = P.out + seg_out;
  const uint16_t *dsrc = P.desc + P.units[sj.first].desc_off;  // 512-aligned
  // descriptor chunk c = bytes [128 c, 128 c + 128): one DMA of 4 bytes per lane
  const uint64_t nchunks = (n + 127) / 128;
  uint64_t issued = 0;
  uint64_t flushed = 0;
  for (uint64_t op = 0; op < n; op += CP_STEP) {
    const uint64_t need = (op >> 7) + 2 < nchunks ? (op >> 7) + 2 : nchunks;
    const uint64_t want = need + CP_AHEAD < nchunks ? need + CP_AHEAD : nchunks;
    while (issued < want) {
      __builtin_amdgcn_global_load_lds(reinterpret_cast<const uint32_t *>(dsrc + issued * 128) + lane,
                                       &sh.desc[(issued * 128) & (CP_DESC_RING - 1)], 4, 0, 0);
      ++issued;
    }
    if (issued - need >= CP_AHEAD)
      __builtin_amdgcn_s_waitcnt(cp_vmcnt(CP_AHEAD));
    else
      __builtin_amdgcn_s_waitcnt(0x0F70);
    // lane j: bytes op + 4 j .. op + 4 j + 3 (bytes past n are never flushed)
    const uint32_t x = (uint32_t)op + 4 * (uint32_t)lane;  // ring / descriptor index (masked)
    const uint64_t dd = *reinterpret_cast<const uint64_t *>(&sh.desc[x & (CP_DESC_RING - 1)]);
    int32_t o0, o1, o2, o3;
    const uint32_t b0 = cp_byte(&sh, op, (uint32_t)dd & 0xFFFF, o0);
    const uint32_t b1 = cp_byte(&sh, op, (uint32_t)(dd >> 16) & 0xFFFF, o1);
    const uint32_t b2 = cp_byte(&sh, op, (uint32_t)(dd >> 32) & 0xFFFF, o2);
    const uint32_t b3 = cp_byte(&sh, op, (uint32_t)(dd >> 48), o3);
    if (__ballot(o0 >= 0 || o1 >= 0 || o2 >= 0 || o3 >= 0) == 0) {
      *reinterpret_cast<uint32_t *>(&sh.ring[x & RING_MASK]) = b0 | (b1 << 8) | (b2 << 16) | (b3 << 24);
    } else {
      // a unit boundary inside this step left references into it: resolve
      // them byte by byte (64-byte sub-steps, pointer jumping)
      for (uint32_t sub = 0; sub < CP_STEP; sub += 64) {
        const uint64_t y = op + sub + (uint64_t)lane;
        const uint32_t d = y < n ? sh.desc[y & (CP_DESC_RING - 1)] : 0x8000u;  // (past n: stale)
        int32_t off;
        uint32_t val = cp_byte(&sh, op, d, off);
        int32_t ptr = -1;
        if (off >= (int32_t)(sub + lane)) off = -1;  // never forward (only stale data could say so)
        if (off >= 0) {
          if ((uint32_t)off < sub)
            val = sh.ring[(op + off) & RING_MASK];  // written by an earlier sub-step
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
        sh.ring[y & RING_MASK] = (uint8_t)val;
        wave_sync();
      }
    }
    wave_sync();
    const uint64_t end = op + CP_STEP < n ? op + CP_STEP : n;
    if (end - flushed >= RS_FLUSH) {
      const uint64_t upto = flushed + RS_FLUSH;
      cp_flush(&sh, out, flushed, upto, lane);
      flushed = upto;
#ifdef ZT_CP_FLUSH_WAIT
      __builtin_amdgcn_s_waitcnt(0x0F70);  // keep vmcnt counting descriptor chunks only
#endif
      // (no wait here: vector memory operations retire in issue order, so the
      // counted descriptor waits above only wait longer with the stores in
      // flight, never shorter)
    }
  }
  wave_sync();
  cp_flush(&sh, out, flushed, n, lane);
  if (lane == 0) P.seg_status[sg] = ZT_OK;
}

}  // namespace

int tokenize_units_dev(const TokParams &p, hipStream_t s) {
  if (p.count == 0) return ZT_OK;
  tokenize_kernel<<<p.count, 64, 0, s>>>(p);
  ZT_HIP(hipGetLastError());
  return ZT_OK;
}

int resolve_segments_dev(const ResolveParams &p, hipStream_t s) {
  if (p.nseg == 0) return ZT_OK;
  expand_kernel<<<p.nunits, 64, 0, s>>>(p);
  ZT_HIP(hipGetLastError());
  copy_kernel<<<p.nseg, 64, 0, s>>>(p);
  ZT_HIP(hipGetLastError());
  return ZT_OK;
}

}  // namespace zt
