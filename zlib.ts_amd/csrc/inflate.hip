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
#include "inflate_common.h"

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

struct InfShared {
  uint8_t ring[RING];
  uint32_t inbuf[IN_RING_WORDS + 4];
  HuffTab lit;
  HuffTab dist;
  uint8_t lens[320];
};


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


// Decode one stream with the calling wave.
template <bool STRICT>
__device__ __forceinline__ void inflate_stream(const InfJob &job, InfResult &res, InfShared *sh) {
  const int lane = threadIdx.x & 63;
  Reader rd;
  rd.init(job.in, job.n, job.start, sh->inbuf, lane);
  Writer wr;
  wr.ring = sh->ring;
  // resume: the history is output position [0, hist_len), never written out
  wr.out = (g_out8 *)(job.out - job.hist_len);
  wr.cap = job.cap + job.hist_len;
  wr.op = job.hist_len;
  wr.flushed = job.hist_len;
  wr.lane = lane;
  for (uint32_t i = lane; i < job.hist_len; i += 64) sh->ring[i & RING_MASK] = job.hist[i];
  wave_sync();
  int status = ZT_OK, detail = 0;
  bool bfinal = false;
  int stop_idx = -1;
  uint64_t si = job.stop_first;
  g_u8 *gin = (g_u8 *)job.in;
  uint32_t v;

  if (job.start > job.n) status = ZT_E_INPUT_BROKEN;
  if (status == ZT_OK && job.start_bit && !rd.template bits<STRICT>((int)job.start_bit, v)) status = ZT_E_INPUT_BROKEN;
  uint64_t blk_bits = job.start * 8 + job.start_bit, blk_op = wr.op;  // end of the last complete block
  while (status == ZT_OK && !bfinal) {
    blk_bits = rd.pos_bits_in();
    blk_op = wr.op;
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
    status = read_tables<STRICT>(rd, sh->lens, lt, dt, btype, lane, detail);
    if (status) break;
    // ---- Huffman block body (src/RawInflate.ts:466-516) ----
    for (;;) {
      if (!STRICT) {
        if (huff_fast(rd, wr, sh, lane) == 0) break;
      }
      wr.op = uni64(wr.op);
      int clen;
      [[maybe_unused]] uint64_t t0 = PROF_T();
      int sym = decode_sym<STRICT>(rd, lt, clen);
      [[maybe_unused]] uint64_t t1 = PROF_T();
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
      [[maybe_unused]] uint64_t t2 = PROF_T();
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
  if (status == ZT_OK) {
    wr.flush(wr.op);
    blk_bits = rd.pos_bits_in();
    blk_op = wr.op;
  } else if (job.resume) {
    wr.flush(blk_op);  // the complete blocks (ring bytes [blk_op - 32 KiB, op) are still held)
  }
  if (lane == 0) {
    res.blk_bits = blk_bits;
    res.blk_op = blk_op;
    res.stop_bits = rd.pos_bits_in();
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
  [[maybe_unused]] const uint64_t t0 = PROF_T();
  [[maybe_unused]] const int lane = threadIdx.x & 63;
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
