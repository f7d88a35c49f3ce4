// inflate.hip -- RFC 1951 raw inflate on the GPU (replaces src/RawInflate.ts
// and src/Huffman.ts).
//
// One wavefront decodes one stream (a batch = one workgroup per stream):
//   * input bits come from a 2 x 64-dword window held in VGPRs (lane i holds
//     dword i); a peek is two v_readlane + a 64-bit funnel shift, and the next
//     256 B are prefetched with one coalesced load while the current ones are
//     consumed;
//   * decode tables are canonical-Huffman LUTs in LDS: a 10-bit primary table
//     (entry = symbol | length << 9) built lane-parallel, longer codes resolved
//     by a 5-step canonical search;
//   * output goes through a 32 KiB LDS history ring; match copies are done by
//     all 64 lanes at once (an overlapping copy with distance d < length reads
//     history[src + (i mod d)], so it needs no serial byte loop); completed
//     4 KiB granules are flushed to HBM with 16-B stores.
// The reader also emulates the reference's byte-refill discipline to report
// its .ip (src/RawInflate.ts:511-514) and whether its over-strict EOF test
// (src/RawInflate.ts:187) would have thrown on this stream.
#include "zt_internal.h"

namespace zt {


#ifdef ZT_INF_PROF
__device__ unsigned long long g_inf_prof[16];
#define PROF_T() ((uint64_t)__builtin_readcyclecounter())
#define PROF_ADD(i, v) (lane == 0 ? (void)atomicAdd(&g_inf_prof[i], (unsigned long long)(v)) : (void)0)
#else
#define PROF_T() 0
#define PROF_ADD(i, v) ((void)0)
#endif

namespace {

constexpr int RING = 32768;
constexpr uint32_t RING_MASK = RING - 1;
constexpr int GRAN = 16384;  // output flush granule (ring holds 32 KiB of history)
constexpr int PRI = 10;

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

// Input bits: the compressed stream is staged through a 16 KiB LDS ring by
// cooperative 8 KiB refills (one wait per 8 KiB of input, never inside the
// per-symbol chain); a 64-bit bit buffer in scalar registers is topped up
// from LDS.  Positions are relative to a 16-byte aligned base below `in`.
constexpr uint32_t IN_RING = 8192;
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

struct InfShared {
  uint8_t ring[RING];
  uint32_t inbuf[IN_RING_WORDS + 4];
  HuffTab lit;
  HuffTab dist;
  uint8_t lens[320];
};

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
    uint32_t r = __brev(v);
    len = 0;
    sym = -1;
    const int ml = (int)uni((uint32_t)t->maxlen);
    for (int l = PRI + 1; l <= ml; ++l) {
      uint32_t c = r >> (32 - l);
      uint32_t k = c - uni(t->first[l]);
      if (k < uni(t->count[l])) {
        len = l;
        sym = (int)uni(t->sorted[uni(t->offs[l]) + k]);
        break;
      }
    }
    if (sym < 0) return ZT_E_INVALID_SYMBOL;  // bits match no code of an incomplete set
  }
  clen = len;
  if (rd.past_end((uint32_t)len)) return ZT_E_INVALID_CODE_LENGTH;
  rd.bb >>= len;
  rd.bc -= len;
  return sym;
}

typedef __attribute__((address_space(1))) uint8_t g_out8;
typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) u32x4_t g_out16;

// copy ring bytes [lo, upto) (clipped to cap) to HBM; out of line and by value
__device__ __attribute__((noinline)) void flush_ring(const uint8_t *ring_, g_out8 *out, uint64_t cap, uint64_t lo,
                                                     uint64_t upto, int lane) {
  typedef __attribute__((address_space(3))) const uint8_t l_u8;
  typedef __attribute__((address_space(3))) const u32x4_t l_u32x4;
  l_u8 *ring = (l_u8 *)ring_;
  const uint64_t hi = upto < cap ? upto : cap;
  if (lo >= hi) return;
  if ((((uintptr_t)out | lo) & 15) == 0) {
    const uint64_t nvec = (hi - lo) >> 4;
    for (uint64_t v = lane; v < nvec; v += 64) {
      const uint64_t p = lo + v * 16;
      *(g_out16 *)(out + p) = *(l_u32x4 *)(ring + (p & RING_MASK));
    }
    for (uint64_t p = lo + nvec * 16 + lane; p < hi; p += 64) out[p] = ring[p & RING_MASK];
  } else {
    for (uint64_t p = lo + lane; p < hi; p += 64) out[p] = ring[p & RING_MASK];
  }
}

struct Writer {
  uint8_t *ring;
  g_out8 *out;
  uint64_t cap;
  uint64_t op;
  uint64_t flushed;  // bytes [0, flushed) are in HBM
  int lane;

  __device__ __forceinline__ void flush(uint64_t upto) {
    flush_ring(ring, out, cap, flushed, upto, lane);
    flushed = upto;
  }
  __device__ __forceinline__ void maybe_flush() {
    if (op - flushed >= GRAN) flush(flushed + GRAN);
  }
};

__device__ __forceinline__ uint32_t fast_mod(uint32_t i, uint32_t d, float inv) {
  uint32_t q = (uint32_t)((float)i * inv);
  int32_t r = (int32_t)i - (int32_t)(q * d);
  if (r < 0) r += (int32_t)d;
  if (r >= (int32_t)d) r -= (int32_t)d;
  return (uint32_t)r;
}


// Huffman block body, fast path (non-strict decoding, >= 16 input bytes left):
// decode entries carry code length, extra-bit count and base value, the bit
// buffer is refilled only when it runs low, and a match copy issues all of its
// ring reads before any write (byte k of a match is history[src + k mod dist],
// which lies before the write cursor), so it costs one LDS round trip.
// Returns 0 at end of block, 1 when the next symbol needs the general path
// (long code, bad symbol or distance, end of input near); state is left at a
// symbol boundary.
__device__ __forceinline__ int huff_fast(Reader &rd, Writer &wr, InfShared *sh, int lane) {
  const uint32_t *lt = sh->lit.pri, *dt = sh->dist.pri;
  uint8_t *ring = sh->ring;
  // all decode state is wave-uniform: pin it to scalar registers
  uint64_t bb = uni64(rd.bb), ip = uni64(rd.ip), op = uni64(wr.op);
  uint32_t bc = uni(rd.bc);
  uint64_t flushed = uni64(wr.flushed);
  const uint64_t hi = uni64(rd.hi);
  const uint64_t ip_end = hi > 16 ? hi - 16 : 0;
  uint64_t fill = uni64(rd.fill);
  // bits in bb come from bytes below ip; the general path may have buffered
  // bits past the end of the input (read as zeros)
  if (ip > ip_end) return 1;
  int ret = 1;
  for (;;) {
    if (bc < 32) {
      if (ip > ip_end) break;
      if (ip + 16 > fill) {
        refill_half_ring(rd.abase, rd.inbuf, rd.lo, hi, fill, lane);
        fill += IN_HALF;
      }
      bb |= rd.ld64(ip) << bc;
      ip += (63 - bc) >> 3;
      bc |= 56;
    }
    const uint32_t e = uni(lt[(uint32_t)bb & ((1u << PRI) - 1)]);
    const uint32_t cl = e & 15;
    const uint32_t sym = (e >> 8) & 511;
    if (sym < 256 && cl) {  // literal (every lane stores the same byte)
      bb >>= cl;
      bc -= cl;
      ring[op & RING_MASK] = (uint8_t)sym;
      op++;
      if (op - flushed >= GRAN) {
        wave_sync();
        wr.flushed = flushed;
        wr.flush(flushed + GRAN);
        flushed += GRAN;
      }
      continue;
    }
    if (sym == 256 && cl) {
      bb >>= cl;
      bc -= cl;
      ret = 0;
      break;
    }
    if (cl == 0) break;  // long code: general path
    // length
    const uint64_t bb0 = bb, ip0 = ip;  // refills only append: (bb0, bc0, ip0) stays valid
    const uint32_t bc0 = bc;
    uint32_t ex = (e >> 4) & 15;
    uint32_t length = (e >> 17) + (((uint32_t)bb >> cl) & ((1u << ex) - 1));
    bb >>= cl + ex;
    bc -= cl + ex;
    if (bc < 28) {
      if (ip > ip_end) {
        bb = bb0;  // general path redoes this symbol
        bc = bc0;
        break;
      }
      if (ip + 16 > fill) {
        refill_half_ring(rd.abase, rd.inbuf, rd.lo, hi, fill, lane);
        fill += IN_HALF;
      }
      bb |= rd.ld64(ip) << bc;
      ip += (63 - bc) >> 3;
      bc |= 56;
    }
    const uint32_t d = uni(dt[(uint32_t)bb & ((1u << PRI) - 1)]);
    const uint32_t dcl = d & 15;
    const uint32_t dsym = (d >> 8) & 511;
    ex = (d >> 4) & 15;
    const uint32_t dist = (d >> 17) + (((uint32_t)bb >> dcl) & ((1u << ex) - 1));
    if (dcl == 0 || dsym >= 30 || dist > op) {
      bb = bb0;  // general path redoes this symbol (and reports the error)
      bc = bc0;
      ip = ip0;
      break;
    }
    bb >>= dcl + ex;
    bc -= dcl + ex;
    // copy: lane handles bytes lane + 64 g
    const uint64_t src = op - dist;
    const uint32_t ng = (length + 63) >> 6;
    uint32_t v[5];
    if (dist >= length) {
#pragma unroll
      for (int g = 0; g < 5; ++g)
        if (g < (int)ng) v[g] = ring[(src + g * 64 + lane) & RING_MASK];
    } else {
      const float inv = __builtin_amdgcn_rcpf((float)dist);
#pragma unroll
      for (int g = 0; g < 5; ++g)
        if (g < (int)ng) v[g] = ring[(src + fast_mod(g * 64 + lane, dist, inv)) & RING_MASK];
    }
#pragma unroll
    for (int g = 0; g < 5; ++g)
      if (g < (int)ng && (uint32_t)(g * 64 + lane) < length) ring[(op + g * 64 + lane) & RING_MASK] = (uint8_t)v[g];
    op += length;
    if (op - flushed >= GRAN) {
      wave_sync();
      wr.flushed = flushed;
      wr.flush(flushed + GRAN);
      flushed += GRAN;
    }
  }
  wr.flushed = flushed;
  rd.bb = bb;
  rd.bc = bc;
  rd.ip = ip;
  rd.fill = fill;
  wr.op = op;
  wave_sync();
  return ret;
}

__constant__ uint8_t kClOrder[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

// Decode one stream with the calling wave.
template <bool STRICT>
__device__ __forceinline__ void inflate_stream(const InfJob &job, InfResult &res, InfShared *sh) {
  const int lane = threadIdx.x & 63;
  Reader rd;
  rd.init(job.in, job.n, job.start, sh->inbuf, lane);
  Writer wr;
  wr.ring = sh->ring;
  wr.out = (g_out8 *)job.out;
  wr.cap = job.cap;
  wr.op = 0;
  wr.flushed = 0;
  wr.lane = lane;
  int status = ZT_OK, detail = 0;
  bool bfinal = false;
  int stop_idx = -1;
  uint64_t si = job.stop_first;
  g_u8 *gin = (g_u8 *)job.in;
  uint32_t v;

  if (job.start > job.n) status = ZT_E_INPUT_BROKEN;
  while (status == ZT_OK && !bfinal) {
    if (!rd.template bits<STRICT>(3, v)) {
      status = ZT_E_INPUT_BROKEN;
      break;
    }
    bfinal = v & 1;
    uint32_t btype = v >> 1;
    if (btype == 0) {
      // ---- stored block (src/RawInflate.ts:251-318) ----
      // the reference drops the buffered bits: ip is the next byte boundary
      const uint64_t nin = job.n;
      uint64_t p = STRICT ? rd.ip_ref : (rd.pos_bits_in() + 7) >> 3;
      if (p + 1 >= nin) {
        status = ZT_E_STORED_LEN;
        break;
      }
      uint32_t len = (uint32_t)job.in[p] | ((uint32_t)job.in[p + 1] << 8);
      if (p + 3 >= nin) {
        status = ZT_E_STORED_NLEN;
        break;
      }
      p += 4;
      if (p + len > nin) {
        status = ZT_E_INPUT_BROKEN;
        break;
      }
      uint32_t done = 0;
      while (done < len) {
        uint32_t room = GRAN - (uint32_t)(wr.op - wr.flushed);
        uint32_t piece = (len - done) < room ? (len - done) : room;
        for (uint32_t j = lane; j < piece; j += 64) sh->ring[(wr.op + j) & RING_MASK] = gin[p + done + j];
        wave_sync();
        wr.op += piece;
        done += piece;
        wr.maybe_flush();
      }
      rd.ip_ref = p + len;
      rd.seek_byte(p + len);
      if (job.stops && !bfinal) {  // segment decode: stop at the next segment start
        const uint64_t q = p + len;
        while (si < job.stop_count && job.stops[si] < q) ++si;
        if (si < job.stop_count && job.stops[si] == q) {
          stop_idx = (int)si;
          break;
        }
      }
      continue;
    }
    HuffTab *lt = &sh->lit, *dt = &sh->dist;
    if (btype == 1) {
      // fixed tables (RFC 1951 3.2.6)
      for (int s = lane; s < 288; s += 64) sh->lens[s] = s <= 143 ? 8 : s <= 255 ? 9 : s <= 279 ? 7 : 8;
      wave_sync();
      build_table(sh->lens, 288, lt, lane, false);
      for (int s = lane; s < 30; s += 64) sh->lens[s] = 5;
      wave_sync();
      build_table(sh->lens, 30, dt, lane, true);
    } else if (btype == 2) {
      // ---- dynamic header (src/RawInflate.ts:345-400) ----
      uint32_t hlit, hdist, hclen;
      if (!rd.template bits<STRICT>(5, hlit) || !rd.template bits<STRICT>(5, hdist) || !rd.template bits<STRICT>(4, hclen)) {
        status = ZT_E_INPUT_BROKEN;
        break;
      }
      hlit += 257;
      hdist += 1;
      hclen += 4;
      if (lane < 19) sh->lens[lane] = 0;
      wave_sync();
      bool ok = true;
      for (uint32_t i = 0; i < hclen; ++i) {
        if (!rd.template bits<STRICT>(3, v)) {
          ok = false;
          break;
        }
        if (lane == 0) sh->lens[kClOrder[i]] = (uint8_t)v;
      }
      wave_sync();
      if (!ok) {
        status = ZT_E_INPUT_BROKEN;
        break;
      }
      int bst = build_table(sh->lens, 19, dt, lane, false);  // code-length code lives in `dist` for now
      if (bst) {
        status = bst;
        break;
      }
      const uint32_t total = hlit + hdist;
      for (int s = lane; s < 320; s += 64) sh->lens[s] = 0;
      wave_sync();
      uint32_t i = 0, prev = 0;
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
          if (i + k < total) sh->lens[i + k] = (uint8_t)val;
        i += rep;
      }
      wave_sync();
      if (status) break;
      bst = build_table(sh->lens, (int)hlit, lt, lane, false);
      if (!bst) bst = build_table(sh->lens + hlit, (int)hdist, dt, lane, true);
      if (bst) {
        status = bst;
        break;
      }
    } else {
      status = ZT_E_UNKNOWN_BTYPE;
      detail = (int)btype;
      break;
    }
    // ---- Huffman block body (src/RawInflate.ts:466-516) ----
    for (;;) {
      if (!STRICT) {
        if (huff_fast(rd, wr, sh, lane) == 0) break;
      }
      wr.op = uni64(wr.op);
      int clen;
      uint64_t t0 = PROF_T();
      int sym = decode_sym<STRICT>(rd, lt, clen);
      uint64_t t1 = PROF_T();
      PROF_ADD(0, t1 - t0);
      PROF_ADD(8, 1);
      if (sym < 0) {
        status = sym;
        detail = clen;
        break;
      }
      if (sym < 256) {
        if (lane == 0) sh->ring[wr.op & RING_MASK] = (uint8_t)sym;
        wr.op++;
        if (wr.op - wr.flushed >= GRAN) {
          wave_sync();
          wr.maybe_flush();
        }
        PROF_ADD(1, PROF_T() - t1);
        continue;
      }
      if (sym == 256) break;
      const uint32_t ls = uni((uint32_t)(sym - 257));  // 286/287 decode as length 258, like the reference
      uint32_t length = len_base(ls);
      const uint32_t lx = len_extra(ls);
      if (lx) {
        if (!rd.template bits<STRICT>((int)lx, v)) { status = ZT_E_INPUT_BROKEN; break; }
        length += v;
      }
      int ds = decode_sym<STRICT>(rd, dt, clen);
      if (ds < 0) {
        status = ds;
        detail = clen;
        break;
      }
      if (ds >= 30) {
        status = ZT_E_INVALID_SYMBOL;
        break;
      }
      const uint32_t dsu = uni((uint32_t)ds);
      uint32_t dist = dist_base(dsu);
      const uint32_t dx = dist_extra(dsu);
      if (dx) {
        if (!rd.template bits<STRICT>((int)dx, v)) { status = ZT_E_INPUT_BROKEN; break; }
        dist += v;
      }
      if (dist > wr.op) {
        status = ZT_E_INVALID_DISTANCE;
        break;
      }
      // parallel copy: byte i comes from history[src + (i mod dist)]
      uint64_t t2 = PROF_T();
      PROF_ADD(2, t2 - t1);
      PROF_ADD(9, 1);
      PROF_ADD(10, length);
      wave_sync();
      const uint64_t src = wr.op - dist;
      const float inv = 1.0f / (float)dist;
      for (uint32_t b0 = 0; b0 < length; b0 += 64) {
        uint32_t i = b0 + lane;
        uint8_t byte = 0;
        if (i < length) {
          uint32_t k = dist >= length ? i : fast_mod(i, dist, inv);
          byte = sh->ring[(src + k) & RING_MASK];
        }
        wave_sync();
        if (i < length) sh->ring[(wr.op + i) & RING_MASK] = byte;
        wave_sync();
      }
      wr.op += length;
      wr.maybe_flush();
      PROF_ADD(3, PROF_T() - t2);
    }
    if (status) break;
    // give back whole unread bytes (src/RawInflate.ts:511-514)
    rd.ip_ref = (rd.pos_bits_in() + 7) >> 3;
  }
  wave_sync();
  if (status == ZT_OK) wr.flush(wr.op);
  if (lane == 0) {
    res.out_len = wr.op;
    res.end_ip = STRICT ? rd.ip_ref : (rd.pos_bits_in() + 7) >> 3;
    res.status = status;
    res.detail = detail;
    res.strict_fail = rd.strict_fail;
    res.stop_idx = stop_idx;
  }
}

__global__ __launch_bounds__(64) void inflate_batch_kernel(const InfJob *__restrict__ jobs,
                                                           InfResult *__restrict__ results, int count) {
  __shared__ InfShared sh;
  const int j = blockIdx.x;
  if (j >= count) return;
  InfJob job = jobs[j];
  InfResult res;
  const uint64_t t0 = PROF_T();
  const int lane = threadIdx.x & 63;
  if (job.strict)
    inflate_stream<true>(job, res, &sh);
  else
    inflate_stream<false>(job, res, &sh);
  PROF_ADD(4, PROF_T() - t0);
  if ((threadIdx.x & 63) == 0) results[j] = res;
}

}  // namespace

#ifdef ZT_INF_PROF
extern "C" int zt_debug_inflate_prof(unsigned long long *out) {
  hipMemcpyFromSymbol(out, HIP_SYMBOL(g_inf_prof), sizeof(unsigned long long) * 16);
  unsigned long long z[16] = {};
  hipMemcpyToSymbol(HIP_SYMBOL(g_inf_prof), z, sizeof z);
  return 0;
}
#endif

int inflate_jobs_dev(const InfJob *d_jobs, InfResult *d_res, int count, hipStream_t s) {
  if (count <= 0) return ZT_OK;
  inflate_batch_kernel<<<count, 64, 0, s>>>(d_jobs, d_res, count);
  ZT_HIP(hipGetLastError());
  return ZT_OK;
}

}  // namespace zt
