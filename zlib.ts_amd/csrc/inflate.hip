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


namespace {

constexpr int RING = 32768;
constexpr uint32_t RING_MASK = RING - 1;
constexpr int GRAN = 4096;
constexpr int PRI = 10;
constexpr uint16_t T_LONG = 0xFFFF;

struct HuffTab {
  uint16_t pri[1 << PRI];
  uint16_t sorted[320];
  uint32_t first[16];
  uint32_t count[16];
  uint32_t offs[16];
  uint32_t running[16];
  int maxlen;
  int status;
};

struct InfShared {
  uint8_t ring[RING];
  HuffTab lit;
  HuffTab dist;
  uint8_t lens[320];
};

__device__ __forceinline__ uint32_t uni(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }

__device__ __forceinline__ uint64_t lanemask_lt(int lane) { return (lane == 0) ? 0ull : (~0ull >> (64 - lane)); }

// Build a canonical decode table from `n` code lengths in s->lens[off..off+n).
// Returns 0, or ZT_E_BAD_TREE for an over-subscribed length set.
__device__ int build_table(const uint8_t *lens, int n, HuffTab *t, int lane) {
  if (lane < 16) {
    t->count[lane] = 0;
    t->running[lane] = 0;
  }
  __syncthreads();
  for (int s = lane; s < n; s += 64) {
    int l = lens[s];
    if (l) atomicAdd(&t->count[l], 1u);
  }
  __syncthreads();
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
  __syncthreads();
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
    __syncthreads();
    if (l && below == 0) t->running[l] += __popcll(peers);
    __syncthreads();
  }
  // primary table: entry e decodes the code whose bits (first bit = bit 0 of e)
  // are a prefix of e
  const int ml = t->maxlen < PRI ? t->maxlen : PRI;
  for (int e = lane; e < (1 << PRI); e += 64) {
    uint32_t r = __brev((uint32_t)e);
    uint16_t ent = T_LONG;
    for (int l = 1; l <= ml; ++l) {
      uint32_t c = r >> (32 - l);
      uint32_t k = c - t->first[l];
      if (k < t->count[l]) {
        ent = (uint16_t)(t->sorted[t->offs[l] + k] | (l << 9));
        break;
      }
    }
    t->pri[e] = ent;
  }
  __syncthreads();
  return t->status;
}

struct Reader {
  const uint8_t *in;
  const uint32_t *abase;  // 4-byte aligned base
  uint32_t boff;          // in - abase (bytes)
  uint64_t n;             // input length
  uint64_t nbits;         // 8 * n
  uint64_t ndw;           // dwords with at least one valid byte
  uint64_t bitpos;        // consumed bits, relative to `in`
  uint64_t wbase;         // first dword of win0
  uint32_t win0, win1;
  uint64_t ip_ref;        // reference's ip
  int strict_fail;
  int strict;
  int lane;

  __device__ uint32_t load_dw(uint64_t k) const {
    if (k >= ndw) return 0;
    uint32_t v = abase[k];
    // zero the bytes outside [boff, boff + n)
    uint64_t b0 = k * 4;
    uint64_t lo = boff, hi = boff + n;
    if (b0 < lo || b0 + 4 > hi) {
      uint32_t m = 0;
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (b0 + j >= lo && b0 + j < hi) m |= 0xFFu << (8 * j);
      v &= m;
    }
    return v;
  }
  __device__ void reload(uint64_t dw) {
    wbase = dw;
    win0 = load_dw(dw + lane);
    win1 = load_dw(dw + 64 + lane);
  }
  __device__ void init(const uint8_t *p, uint64_t len, uint64_t start, int ln) {
    in = p;
    lane = ln;
    uintptr_t a = reinterpret_cast<uintptr_t>(p);
    abase = reinterpret_cast<const uint32_t *>(a & ~uintptr_t(3));
    boff = (uint32_t)(a & 3);
    n = len;
    nbits = len * 8;
    ndw = (boff + len + 3) / 4;
    bitpos = start * 8;
    ip_ref = start;
    strict_fail = 0;
    reload((bitpos + 8 * boff) >> 5);
  }
  // 32 bits starting at bitpos (bits past the end read as 0)
  __device__ uint32_t peek() {
    uint64_t bp = bitpos + 8ull * boff;
    uint64_t dw = bp >> 5;
    uint64_t d = dw - wbase;
    if (d >= 64) {
      if (d < 128) {
        win0 = win1;
        wbase += 64;
        win1 = load_dw(wbase + 64 + lane);
      } else {
        reload(dw);
      }
      d = dw - wbase;
    }
    int di = (int)d;
    uint32_t lo = di < 64 ? __builtin_amdgcn_readlane(win0, di) : __builtin_amdgcn_readlane(win1, di - 64);
    uint32_t hi = di + 1 < 64 ? __builtin_amdgcn_readlane(win0, di + 1) : __builtin_amdgcn_readlane(win1, di - 63);
    uint64_t v = (((uint64_t)hi << 32) | lo) >> (bp & 31);
    return (uint32_t)v;
  }
  // readBits(nb) with the reference's EOF test; returns false past the end
  __device__ bool bits(int nb, uint32_t &out) {
    int64_t bbl = (int64_t)(ip_ref * 8) - (int64_t)bitpos;
    int64_t need = ((int64_t)nb - bbl + 7) >> 3;
    if ((int64_t)ip_ref + need >= (int64_t)n) {
      strict_fail = 1;
      if (strict) return false;
    }
    uint64_t want = (bitpos + nb + 7) >> 3;
    if (want > ip_ref) ip_ref = want;
    if (bitpos + nb > nbits) return false;
    out = nb ? (peek() & ((1u << nb) - 1)) : 0;
    bitpos += nb;
    return true;
  }
  // note the reference's refill for a readCodeByTable with this maxlen
  __device__ void code_refill(int maxlen) {
    uint64_t want = (bitpos + maxlen + 7) >> 3;
    if (want > n) want = n;
    if (want > ip_ref) ip_ref = want;
  }
};

// Decode one symbol; returns symbol or a negative status; *clen = code length
__device__ __forceinline__ int decode_sym(Reader &rd, const HuffTab *t, int &clen) {
  rd.code_refill(t->maxlen);
  uint32_t v = rd.peek();
  uint32_t e = uni(t->pri[v & ((1u << PRI) - 1)]);
  int len, sym;
  if (e != T_LONG) {
    len = (int)(e >> 9);
    sym = (int)(e & 511);
  } else {
    uint32_t r = __brev(v);
    len = 0;
    sym = -1;
    for (int l = PRI + 1; l <= t->maxlen; ++l) {
      uint32_t c = r >> (32 - l);
      uint32_t k = c - t->first[l];
      if (k < t->count[l]) {
        len = l;
        sym = t->sorted[t->offs[l] + k];
        break;
      }
    }
    sym = (int)uni((uint32_t)sym);
    len = (int)uni((uint32_t)len);
    if (sym < 0) return ZT_E_INVALID_SYMBOL;  // bits match no code of an incomplete set
  }
  clen = len;
  if (rd.bitpos + (uint64_t)len > rd.nbits) return ZT_E_INVALID_CODE_LENGTH;
  rd.bitpos += len;
  return sym;
}

struct Writer {
  uint8_t *ring;
  uint8_t *out;
  uint64_t cap;
  uint64_t op;
  uint64_t flushed;  // bytes [0, flushed) are in HBM
  int lane;

  // copy ring bytes [flushed, upto) to HBM (upto - flushed <= RING)
  __device__ void flush(uint64_t upto) {
    uint64_t lo = flushed, hi = upto < cap ? upto : cap;
    if (lo < hi) {
      bool aligned = ((reinterpret_cast<uintptr_t>(out) | lo) & 15) == 0;
      if (aligned) {
        uint64_t nvec = (hi - lo) >> 4;
        for (uint64_t v = lane; v < nvec; v += 64) {
          uint64_t p = lo + v * 16;
          uint4 x = *reinterpret_cast<const uint4 *>(ring + (p & RING_MASK));
          *reinterpret_cast<uint4 *>(out + p) = x;
        }
        for (uint64_t p = lo + nvec * 16 + lane; p < hi; p += 64) out[p] = ring[p & RING_MASK];
      } else {
        for (uint64_t p = lo + lane; p < hi; p += 64) out[p] = ring[p & RING_MASK];
      }
    }
    flushed = upto;
  }
  __device__ void maybe_flush() {
    uint64_t g = op & ~(uint64_t)(GRAN - 1);
    if (g > flushed) flush(g);
  }
};

__device__ __forceinline__ uint32_t fast_mod(uint32_t i, uint32_t d, float inv) {
  uint32_t q = (uint32_t)((float)i * inv);
  int32_t r = (int32_t)i - (int32_t)(q * d);
  if (r < 0) r += (int32_t)d;
  if (r >= (int32_t)d) r -= (int32_t)d;
  return (uint32_t)r;
}

__constant__ uint16_t kLenBase[31] = {3,  4,  5,  6,  7,  8,  9,  10, 11,  13,  15,  17,  19,  23, 27, 31,
                                      35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 258, 258, 258};
__constant__ uint8_t kLenExtra[31] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2,
                                      3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0, 0, 0};
__constant__ uint16_t kDistBase[30] = {1,    2,    3,    4,    5,    7,    9,    13,    17,    25,
                                       33,   49,   65,   97,   129,  193,  257,  385,   513,   769,
                                       1025, 1537, 2049, 3073, 4097, 6145, 8193, 12289, 16385, 24577};
__constant__ uint8_t kDistExtra[30] = {0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6,
                                       6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13};
__constant__ uint8_t kClOrder[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

// Decode one stream with the calling wave.
__device__ void inflate_stream(const InfJob &job, InfResult &res, InfShared *sh) {
  const int lane = threadIdx.x & 63;
  Reader rd;
  rd.init(job.in, job.n, job.start, lane);
  rd.strict = job.strict;
  Writer wr;
  wr.ring = sh->ring;
  wr.out = job.out;
  wr.cap = job.cap;
  wr.op = 0;
  wr.flushed = 0;
  wr.lane = lane;
  int status = ZT_OK, detail = 0;
  bool bfinal = false;
  uint32_t v;

  if (job.start > job.n) status = ZT_E_INPUT_BROKEN;
  while (status == ZT_OK && !bfinal) {
    if (!rd.bits(3, v)) {
      status = ZT_E_INPUT_BROKEN;
      break;
    }
    bfinal = v & 1;
    uint32_t btype = v >> 1;
    if (btype == 0) {
      // ---- stored block (src/RawInflate.ts:251-318) ----
      uint64_t p = rd.ip_ref;  // reference drops the buffered bits: ip is byte aligned
      if (p + 1 >= rd.n) {
        status = ZT_E_STORED_LEN;
        break;
      }
      uint32_t len = (uint32_t)job.in[p] | ((uint32_t)job.in[p + 1] << 8);
      if (p + 3 >= rd.n) {
        status = ZT_E_STORED_NLEN;
        break;
      }
      p += 4;
      if (p + len > rd.n) {
        status = ZT_E_INPUT_BROKEN;
        break;
      }
      uint32_t done = 0;
      while (done < len) {
        uint32_t room = GRAN - (uint32_t)(wr.op & (GRAN - 1));
        uint32_t piece = (len - done) < room ? (len - done) : room;
        for (uint32_t j = lane; j < piece; j += 64) sh->ring[(wr.op + j) & RING_MASK] = job.in[p + done + j];
        __syncthreads();
        wr.op += piece;
        done += piece;
        wr.maybe_flush();
      }
      rd.ip_ref = p + len;
      rd.bitpos = (p + len) * 8;
      continue;
    }
    HuffTab *lt = &sh->lit, *dt = &sh->dist;
    if (btype == 1) {
      // fixed tables (RFC 1951 3.2.6)
      for (int s = lane; s < 288; s += 64) sh->lens[s] = s <= 143 ? 8 : s <= 255 ? 9 : s <= 279 ? 7 : 8;
      __syncthreads();
      build_table(sh->lens, 288, lt, lane);
      for (int s = lane; s < 30; s += 64) sh->lens[s] = 5;
      __syncthreads();
      build_table(sh->lens, 30, dt, lane);
    } else if (btype == 2) {
      // ---- dynamic header (src/RawInflate.ts:345-400) ----
      uint32_t hlit, hdist, hclen;
      if (!rd.bits(5, hlit) || !rd.bits(5, hdist) || !rd.bits(4, hclen)) {
        status = ZT_E_INPUT_BROKEN;
        break;
      }
      hlit += 257;
      hdist += 1;
      hclen += 4;
      if (lane < 19) sh->lens[lane] = 0;
      __syncthreads();
      bool ok = true;
      for (uint32_t i = 0; i < hclen; ++i) {
        if (!rd.bits(3, v)) {
          ok = false;
          break;
        }
        if (lane == 0) sh->lens[kClOrder[i]] = (uint8_t)v;
      }
      __syncthreads();
      if (!ok) {
        status = ZT_E_INPUT_BROKEN;
        break;
      }
      int bst = build_table(sh->lens, 19, dt, lane);  // code-length code lives in `dist` for now
      if (bst) {
        status = bst;
        break;
      }
      const uint32_t total = hlit + hdist;
      for (int s = lane; s < 320; s += 64) sh->lens[s] = 0;
      __syncthreads();
      uint32_t i = 0, prev = 0;
      while (i < total) {
        int clen;
        int sym = decode_sym(rd, dt, clen);
        if (sym < 0) {
          status = sym;
          detail = clen;
          break;
        }
        uint32_t rep, val;
        if (sym == 16) {
          if (!rd.bits(2, v)) { status = ZT_E_INPUT_BROKEN; break; }
          rep = 3 + v;
          val = prev;
        } else if (sym == 17) {
          if (!rd.bits(3, v)) { status = ZT_E_INPUT_BROKEN; break; }
          rep = 3 + v;
          val = 0;
          prev = 0;
        } else if (sym == 18) {
          if (!rd.bits(7, v)) { status = ZT_E_INPUT_BROKEN; break; }
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
      __syncthreads();
      if (status) break;
      bst = build_table(sh->lens, (int)hlit, lt, lane);
      if (!bst) bst = build_table(sh->lens + hlit, (int)hdist, dt, lane);
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
      int clen;
      int sym = decode_sym(rd, lt, clen);
      if (sym < 0) {
        status = sym;
        detail = clen;
        break;
      }
      if (sym < 256) {
        if (lane == 0) sh->ring[wr.op & RING_MASK] = (uint8_t)sym;
        wr.op++;
        if ((wr.op & (GRAN - 1)) == 0) {
          __syncthreads();
          wr.maybe_flush();
        }
        continue;
      }
      if (sym == 256) break;
      const int ls = sym - 257;  // 286/287 decode as length 258, like the reference's tables
      uint32_t length = kLenBase[ls];
      if (kLenExtra[ls]) {
        if (!rd.bits(kLenExtra[ls], v)) { status = ZT_E_INPUT_BROKEN; break; }
        length += v;
      }
      int ds = decode_sym(rd, dt, clen);
      if (ds < 0) {
        status = ds;
        detail = clen;
        break;
      }
      if (ds >= 30) {
        status = ZT_E_INVALID_SYMBOL;
        break;
      }
      uint32_t dist = kDistBase[ds];
      if (kDistExtra[ds]) {
        if (!rd.bits(kDistExtra[ds], v)) { status = ZT_E_INPUT_BROKEN; break; }
        dist += v;
      }
      if (dist > wr.op) {
        status = ZT_E_INVALID_DISTANCE;
        break;
      }
      // parallel copy: byte i comes from history[src + (i mod dist)]
      __syncthreads();
      const uint64_t src = wr.op - dist;
      const float inv = 1.0f / (float)dist;
      for (uint32_t b0 = 0; b0 < length; b0 += 64) {
        uint32_t i = b0 + lane;
        uint8_t byte = 0;
        if (i < length) {
          uint32_t k = dist >= length ? i : fast_mod(i, dist, inv);
          byte = sh->ring[(src + k) & RING_MASK];
        }
        __syncthreads();
        if (i < length) sh->ring[(wr.op + i) & RING_MASK] = byte;
        __syncthreads();
      }
      wr.op += length;
      wr.maybe_flush();
    }
    if (status) break;
    // give back whole unread bytes (src/RawInflate.ts:511-514)
    rd.ip_ref = (rd.bitpos + 7) >> 3;
  }
  __syncthreads();
  if (status == ZT_OK) wr.flush(wr.op);
  if (lane == 0) {
    res.out_len = wr.op;
    res.end_ip = rd.ip_ref;
    res.status = status;
    res.detail = detail;
    res.strict_fail = rd.strict_fail;
  }
}

__global__ __launch_bounds__(64) void inflate_batch_kernel(const InfJob *__restrict__ jobs,
                                                           InfResult *__restrict__ results, int count) {
  __shared__ InfShared sh;
  const int j = blockIdx.x;
  if (j >= count) return;
  InfJob job = jobs[j];
  InfResult res;
  inflate_stream(job, res, &sh);
  if ((threadIdx.x & 63) == 0) results[j] = res;
}

}  // namespace

int inflate_jobs_dev(const InfJob *d_jobs, InfResult *d_res, int count, hipStream_t s) {
  if (count <= 0) return ZT_OK;
  inflate_batch_kernel<<<count, 64, 0, s>>>(d_jobs, d_res, count);
  ZT_HIP(hipGetLastError());
  return ZT_OK;
}

}  // namespace zt
