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

__global__ __launch_bounds__(64) void tokenize_kernel(TokParams P) {
  __shared__ TokShared sh;
  const uint32_t u = blockIdx.x;
  const int lane = threadIdx.x & 63;
  const TokJob job = P.jobs[u];
  const uint64_t n = P.n;
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
      status = tok_huffman(rd, &sh.lit, &sh.dist, to, op);
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

__device__ __forceinline__ uint32_t incl_scan(uint32_t x, int lane) {
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const uint32_t y = __shfl_up(x, off, 64);
    if (lane >= off) x += y;
  }
  return x;
}

struct ResolveShared {
  uint8_t ring[RING];
  uint32_t mark[64];
};

__device__ __forceinline__ uint32_t tok_len(uint32_t t) { return (t >> 16) ? (t >> 16) : 1u; }

__global__ __launch_bounds__(64) void resolve_kernel(ResolveParams P) {
  __shared__ ResolveShared sh;
  const uint32_t sg = blockIdx.x;
  const int lane = threadIdx.x & 63;
  const SegJob sj = P.segs[sg];
  const uint64_t seg_out = P.units[sj.first].out_off;
  uint8_t *out = P.out + seg_out;
  sh.mark[lane] = 0;
  uint32_t seq = 0;
  uint64_t op = 0;  // segment-relative output position
  int status = ZT_OK;
  for (uint32_t k = 0; k < sj.count && status == ZT_OK; ++k) {
    const ChainUnit cu = P.units[sj.first + k];
    const uint32_t *tk = P.tokens + cu.tok_off;
    const uint32_t ntok = cu.ntok;
    // tokens [base, base + 256) live in A, B, C, D (lane i: token base + 64 r + i)
    uint32_t base = 0;
    uint32_t A = (uint32_t)lane < ntok ? tk[lane] : 0u;
    uint32_t B = 64u + lane < ntok ? tk[64 + lane] : 0u;
    uint32_t C = 128u + lane < ntok ? tk[128 + lane] : 0u;
    uint32_t D = 192u + lane < ntok ? tk[192 + lane] : 0u;
    uint32_t cur = 0, rem = 0;
    const uint64_t op_unit = op;
    while (cur < ntok) {
      const uint32_t c = cur - base;  // 0..63
      const uint32_t si = c + (uint32_t)lane;
      const uint32_t ta = bperm(A, si & 63), tb = bperm(B, si & 63);
      const bool valid = cur + (uint32_t)lane < ntok;
      const uint32_t t = si < 64 ? ta : tb;
      const uint32_t len = valid ? tok_len(t) : 0u;
      const uint32_t S = incl_scan(len, lane);
      const uint32_t total = uni(__builtin_amdgcn_readlane(S, 63)) - rem;
      const uint32_t W = total < 64 ? total : 64;
      // token i + 1 starts at S_i - rem inside the window
      ++seq;
      const int32_t p = (int32_t)S - (int32_t)rem;
      if (valid && p > 0 && p < 64) sh.mark[p] = seq;
      wave_sync();
      const uint64_t starts = __ballot(sh.mark[lane] == seq);
      const uint32_t ti = __popcll(starts & (~0ull >> (63 - lane)));  // token of byte `lane`
      const uint32_t tj = bperm(t, ti);
      uint32_t val = 0;
      bool bad = false;
      int32_t ptr = -1;
      if ((uint32_t)lane < W) {
        if ((tj >> 16) == 0) {
          val = tj & 0xFF;
        } else {
          const uint32_t dist = tj & 0xFFFF;
          const uint64_t pos = op + (uint64_t)lane;
          if (dist > pos) {
            bad = true;  // reaches behind the segment start
          } else {
            const uint64_t src = pos - dist;
            if (src >= op)
              ptr = (int32_t)(src - op);
            else
              val = sh.ring[src & RING_MASK];
          }
        }
      }
      if (__ballot(bad)) {
        status = ZT_E_INVALID_DISTANCE;
        break;
      }
      // in-window references: pointer jumping (a source lane precedes its reader)
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
      if ((uint32_t)lane < W) {
        sh.ring[(op + lane) & RING_MASK] = (uint8_t)val;
        out[op + lane] = (uint8_t)val;
      }
      wave_sync();
      op += W;
      // advance past the tokens that end inside this window
      const uint64_t done = __ballot(valid && S <= rem + W);
      const uint32_t kk = (uint32_t)__popcll(done);
      const uint32_t s_last = kk ? uni(__builtin_amdgcn_readlane(S, kk - 1)) : 0u;
      rem = rem + W - s_last;
      cur += kk;
      while (cur - base >= 64) {
        A = B;
        B = C;
        C = D;
        base += 64;
        const uint32_t ix = base + 192 + (uint32_t)lane;
        D = ix < ntok ? tk[ix] : 0u;
      }
    }
    if (op - op_unit != cu.out_len) status = ZT_E_INPUT_BROKEN;
  }
  if (lane == 0) P.seg_status[sg] = status;
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
  resolve_kernel<<<p.nseg, 64, 0, s>>>(p);
  ZT_HIP(hipGetLastError());
  return ZT_OK;
}

}  // namespace zt
