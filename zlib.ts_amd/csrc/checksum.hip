// checksum.hip -- CRC-32 and Adler-32 over device-resident bytes, fused in
// one HBM pass (replaces src/CRC32.ts:25-47 and src/Adler32.ts:28-48).
//
// Decomposition (HBM-bound byte work; no MFMA):
//   * the input is cut into CK_SEG-byte segments (1 MiB), one 256-thread
//     workgroup each (grid-stride), CK_SEG / 4 contiguous bytes per wave;
//   * loads are coalesced: each wave instruction reads 1 KiB contiguous, lane
//     l the 16 bytes at 16 l; a row is 8 such loads (8 KiB per wave), so a
//     lane holds 32 words per row, word j = 4 q + w at 1024 q + 16 l + 4 w;
//   * CRC-32, table-free and bit-sliced: the lane runs 32 streams (stream j =
//     word j of every row) in 32 registers P[0..31], P[b] holding state bit
//     b of all 32 streams.  Per row the 32 data words are transposed into the
//     same form (16 v_perm_b32 + 96 v_bfi_b32 pairs' worth of selects) and
//     the streams advance by one row: P <- A P ^ D, A = multiplication by
//     x^(8 * 8192) mod P, a constant 32 x 32 GF(2) matrix unrolled at compile
//     time into 3-input XORs (v_bitop3_b32) -- about 4 VALU per byte, no
//     LDS; the 32 streams then fold pairwise into one (streams 16 apart are
//     4 KiB apart: P <- M P ^ (P >> 16), then 8, 4, 2, 1) and the lane's CRC
//     moves to the segment end by one multiplication;
//   * Adler: v_dot4_u32_u8 sums per 16-byte piece, positions weighted from
//     the piece's place in the segment;
//   * per-lane results are merged with polynomial shifts (CRC) and weighted
//     sums (Adler) inside the workgroup; segments merge by atomics and the
//     last workgroup to finish writes the result (batch: a small kernel).
//     Ragged first / last segments take a byte-wise per-thread-slice path
//     (slice-by-8 through nibble tables in LDS).
// Algorithmic bytes per unit: N input bytes read.
#include <vector>

#include "zt_internal.h"

namespace zt {

namespace {

#ifndef ZT_CK_THREADS
#define ZT_CK_THREADS 256
#endif
#ifndef ZT_CK_ROWS
#define ZT_CK_ROWS 32  // 8 KiB rows per wave: a segment is 4 waves x ZT_CK_ROWS x 8 KiB (16: 0.25 ms per GiB, 32: 0.23)
#endif
#ifndef ZT_CK_DEPTH
#define ZT_CK_DEPTH 2  // rows of loads in registers (3: the next two rows in flight)
#endif
#ifndef ZT_CK_MINW
#define ZT_CK_MINW 2  // waves per SIMD the register allocation must allow (4: 128 VGPRs, spills)
#endif
constexpr int CK_THREADS = ZT_CK_THREADS;
constexpr int CK_ROWS = ZT_CK_ROWS;
constexpr int CK_ROW = 8192;                                   // bytes per row (one wave: 8 x 1 KiB loads)
constexpr int CK_WAVE_BYTES = CK_ROWS * CK_ROW;                // contiguous bytes per wave in a whole segment
constexpr size_t CK_SEG = (size_t)CK_WAVE_BYTES * (CK_THREADS / 64);
constexpr int CK_SLICE = (int)(CK_SEG / CK_THREADS);          // bytes per thread (ragged segments)
// the ragged path's u32 Adler s2 of one slice: 255 n (n + 1) / 2 < 2^32
static_assert(CK_SLICE <= 4096, "slice Adler sums overflow");
static_assert(CK_THREADS % 64 == 0 && CK_SLICE % 128 == 0, "geometry");

// batch checksums: segment k of the buffer at frame + off (off 16-byte aligned)
struct CkJob {
  uint64_t off;
  uint64_t len;
  uint64_t k;
};

struct SegResult {
  uint32_t crc;   // raw CRC register (init 0, no final xor) over the segment's bytes
  uint32_t len;   // valid bytes in the segment
  uint32_t s1;    // Adler sums mod 65521 (init 0)
  uint32_t s2;
};

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint4 ld_stream(const uint4 *p) {
  u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(p));
  return make_uint4(v.x, v.y, v.z, v.w);
}

// Nibble table layout in LDS (byte address): position pos (0..23), nibble
// value v, replica r = lane & 31 at (pos >> 1) * 4096 + v * 256 + (pos & 1) *
// 128 + 4 r.  Lane l always reads bank l & 31 (conflict-free), and a lookup's
// address is one v_perm_b32: byte 0 the lane's 4 r, byte 1 the nibble, taken
// from a word whose bytes hold nibbles (a & 0x0F0F0F0F or (a >> 4) & ...);
// the table position is the ds_read's immediate offset.
__device__ __forceinline__ uint32_t nib_index(uint32_t i) {  // LDS word i -> nib_g entry
  const uint32_t pos = ((i >> 10) << 1) | ((i >> 5) & 1u);
  return (pos << 4) + ((i >> 6) & 15u);
}

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  uint32_t r;
  asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}

// the 8 lookups of word a's nibbles in tables P0 .. P0 + 7 (P0 even)
template <int P0>
__device__ __forceinline__ void lut8(uint32_t a, const uint32_t *T, uint32_t lb, uint32_t *t) {
  const uint32_t me = a & 0x0F0F0F0Fu, mo = (a >> 4) & 0x0F0F0F0Fu;
  const char *Tb = reinterpret_cast<const char *>(T);
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const uint32_t sel = 0x0C0C0400u | ((uint32_t)k << 8);
    const uint32_t ae = __builtin_amdgcn_perm(me, lb, sel), ao = __builtin_amdgcn_perm(mo, lb, sel);
    t[2 * k] = *reinterpret_cast<const uint32_t *>(Tb + ae + (P0 / 2 + k) * 4096);
    t[2 * k + 1] = *reinterpret_cast<const uint32_t *>(Tb + ao + (P0 / 2 + k) * 4096 + 128);
  }
}

// One 8-byte CRC step: state xors into the first 4 bytes (reflected slice-by-8).
// lb = 4 * (lane & 31)
__device__ __forceinline__ uint32_t crc_step8(uint32_t c, uint32_t w0, uint32_t w1, const uint32_t *T, uint32_t lb) {
  uint32_t t[16];
  lut8<8>(w1, T, lb, t + 8);
  lut8<0>(c ^ w0, T, lb, t);
  const uint32_t x0 = xor3(t[8], t[9], t[10]), x1 = xor3(t[11], t[12], t[13]), x2 = xor3(t[14], t[15], t[0]);
  const uint32_t x3 = xor3(t[1], t[2], t[3]), x4 = xor3(t[4], t[5], t[6]);
  return xor3(x0, x1, x2) ^ xor3(x3, x4, t[7]);
}

// ---- bit-sliced CRC-32 ----------------------------------------------------
// GF(2) arithmetic of zlib's multmodp convention (x^0 = bit 31), at compile
// time: the matrices below are folded into the instruction stream.
constexpr uint32_t cx_mult(uint32_t a, uint32_t b) {
  uint32_t p = 0;
  for (int i = 31; i >= 0; --i) {
    if ((a >> i) & 1u) p ^= b;
    b = (b & 1u) ? (b >> 1) ^ ZT_CRC_POLY : b >> 1;
  }
  return p;
}
constexpr uint32_t cx_x8n(uint64_t n) {  // x^(8 n) mod P
  uint32_t p = 1u << 31, base = 1u << 23;
  while (n) {
    if (n & 1u) p = cx_mult(base, p);
    base = cx_mult(base, base);
    n >>= 1;
  }
  return p;
}
struct GfMat {
  uint32_t row[32];  // row[b] bit a: bit b of (K * e_a), e_a = the register with only bit a set
};
constexpr GfMat cx_mat(uint32_t K) {
  GfMat m{};
  for (int a = 0; a < 32; ++a) {
    const uint32_t c = cx_mult(K, 1u << a);
    for (int b = 0; b < 32; ++b)
      if ((c >> b) & 1u) m.row[b] |= 1u << a;
  }
  return m;
}

// in[a] for every set bit a of the compile-time mask M, XOR-ed into acc, two
// terms per 3-input XOR (v_bitop3_b32; the transpose's selects are inline asm:
// LLVM otherwise re-associates this XOR network through them and multiplies
// its size by six)
template <uint32_t M, int A = 0>
__device__ __forceinline__ uint32_t xor_terms(const uint32_t (&in)[32], uint32_t acc) {
  if constexpr (A == 32) {
    return acc;
  } else if constexpr (((M >> A) & 1u) == 0) {
    return xor_terms<M, A + 1>(in, acc);
  } else {
    constexpr uint32_t rest = M & ~((2u << A) - 1u);  // set bits above A
    if constexpr (rest == 0) {
      return acc ^ in[A];
    } else {
      constexpr int A2 = __builtin_ctz(rest);
      return xor_terms<M, A2 + 1>(in, __builtin_amdgcn_bitop3_b32(acc, in[A], in[A2], 0x96));
    }
  }
}
template <uint32_t K, int B = 0>
__device__ __forceinline__ void gf_rows(const uint32_t (&in)[32], const uint32_t (&add)[32], uint32_t (&out)[32]) {
  if constexpr (B < 32) {
    constexpr uint32_t M = cx_mat(K).row[B];
    out[B] = xor_terms<M>(in, add[B]);
    gf_rows<K, B + 1>(in, add, out);
  }
}
// out[b] = add[b] ^ (K * stream) bit b: the 32 streams of the planes each
// multiplied by K
template <uint32_t K>
__device__ __forceinline__ void gf_mul_planes(const uint32_t (&in)[32], const uint32_t (&add)[32], uint32_t (&out)[32]) {
  gf_rows<K>(in, add, out);
}

// 32 x 32 bit transpose in place: afterwards w[b] bit j = bit b of the
// former w[j].  Block swaps of 16 and 8 bits by byte permutes, 4, 2, 1 by
// shifts and bit-field selects (v_bfi_b32).
// (builtins, not inline asm: the hazard recognizer then knows them and adds
// no s_nop between dependent ones)
__device__ __forceinline__ uint32_t perm_asm(uint32_t s0, uint32_t s1, uint32_t sel) {
  return __builtin_amdgcn_perm(s0, s1, sel);
}
__device__ __forceinline__ uint32_t bfi_asm(uint32_t m, uint32_t a, uint32_t b) {  // (m & a) | (~m & b)
  return __builtin_amdgcn_bitop3_b32(m, a, b, 0xCA);
}
// rows k and k + S (k & S == 0): bits of the S-wide columns exchanged
template <int S>
__device__ __forceinline__ void swap_stage(uint32_t (&w)[32], uint32_t m) {
#pragma unroll
  for (int k = 0; k < 32; ++k) {
    if ((k & S) == 0) {
      const uint32_t a = w[k], b = w[k + S];
      w[k] = bfi_asm(m, a, b << S);
      w[k + S] = bfi_asm(m, a >> S, b);
    }
  }
}
__device__ __forceinline__ void transpose32(uint32_t (&w)[32]) {
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const uint32_t a = w[k], b = w[k + 16];
    w[k] = perm_asm(b, a, 0x05040100u);       // a.lo16 | b.lo16 << 16
    w[k + 16] = perm_asm(b, a, 0x07060302u);  // a.hi16 | b.hi16 << 16
  }
#pragma unroll
  for (int k0 = 0; k0 < 32; k0 += 16)
#pragma unroll
    for (int k = k0; k < k0 + 8; ++k) {
      const uint32_t a = w[k], b = w[k + 8];
      w[k] = perm_asm(b, a, 0x06020400u);      // bytes a0 b0 a2 b2
      w[k + 8] = perm_asm(b, a, 0x07030501u);  // bytes a1 b1 a3 b3
    }
  swap_stage<4>(w, 0x0F0F0F0Fu);
  swap_stage<2>(w, 0x33333333u);
  swap_stage<1>(w, 0x55555555u);
}

__device__ __forceinline__ uint32_t crc_byte(uint32_t c, uint32_t b) {
  c ^= b;
#pragma unroll
  for (int k = 0; k < 8; ++k) c = (c & 1) ? (c >> 1) ^ ZT_CRC_POLY : c >> 1;
  return c;
}

// Adler over one 16-byte piece: s2 += 16*s1 + weighted(piece); s1 += sum(piece)
__device__ __forceinline__ void adler16(uint32_t &s1, uint32_t &s2, uint4 v) {
  uint32_t w = __builtin_amdgcn_udot4(v.x, 0x0D0E0F10u, 0u, false);
  w = __builtin_amdgcn_udot4(v.y, 0x090A0B0Cu, w, false);
  w = __builtin_amdgcn_udot4(v.z, 0x05060708u, w, false);
  w = __builtin_amdgcn_udot4(v.w, 0x01020304u, w, false);
  uint32_t s = __builtin_amdgcn_udot4(v.x, 0x01010101u, 0u, false);
  s = __builtin_amdgcn_udot4(v.y, 0x01010101u, s, false);
  s = __builtin_amdgcn_udot4(v.z, 0x01010101u, s, false);
  s = __builtin_amdgcn_udot4(v.w, 0x01010101u, s, false);
  s2 += (s1 << 4) + w;
  s1 += s;
}

// x^(8 n) * c mod P from the base-64 digit tables (ZT_CRC_DIGITS digits;
// longer shifts finish with the squares table)
__device__ inline uint32_t shift_bytes(const uint32_t *__restrict__ dig, const uint32_t *__restrict__ x2n,
                                       uint64_t n, uint32_t c) {
#pragma unroll
  for (int d = 0; d < ZT_CRC_DIGITS; ++d) {
    const uint32_t v = (uint32_t)(n >> (6 * d)) & 63u;
    if (v) c = multmodp(dig[d * 64 + v], c);
  }
  const uint64_t rest = n >> (6 * ZT_CRC_DIGITS);
  if (rest) c = multmodp(x2nmodp(x2n, rest, 3 + 6 * ZT_CRC_DIGITS), c);
  return c;
}

// One buffer's merge inside checksum_segments: every workgroup adds its
// segments' (already end-shifted) results to `acc` by atomics, workgroup 0
// adds the caller's initial CRC shifted over the whole buffer, and the
// workgroup that arrives last writes the final values and leaves `acc`
// zeroed for the next call.  One accumulator per device context: correctness
// rests on every caller of checksums_dev synchronising the launch stream
// before it releases the context mutex (zt_dev_checksums waits on its stream,
// the container calls on c->aux through AuxWait), so no two launches share
// `acc` at once; an asynchronous caller would need its own accumulator.
// A separate one-workgroup finish kernel cost 6 us + its launch per call.
struct CkFinish {
  CkAcc *acc;  // null: batch mode (per-segment results to `out`)
  uint32_t *result;
  uint64_t n;
  uint32_t crc_in, adler_in;
};

template <bool DO_CRC, bool DO_ADLER>
__global__ __launch_bounds__(CK_THREADS, ZT_CK_MINW) void checksum_segments(const uint8_t *__restrict__ frame0, size_t lo0,
                                                                 size_t hi0, size_t nseg,
                                                                 const uint32_t *__restrict__ nib_g,
                                                                 const uint32_t *__restrict__ x2n_g,
                                                                 const uint32_t *__restrict__ shift_g,
                                                                 SegResult *__restrict__ out,
                                                                 const CkJob *__restrict__ jobs, CkFinish fin) {
  // 32 KiB of replicated nibble tables + the combine scratch
  __shared__ uint32_t T[DO_CRC ? 256 * 32 : 1];  // nibble positions 0..15 (ragged slices only)
  __shared__ uint32_t x2n[32];
  __shared__ uint32_t red_c[1];
  __shared__ unsigned long long red_a[CK_THREADS / 64][2];
  __shared__ uint32_t red_w[CK_THREADS / 64];

  const int tid = threadIdx.x;
  const uint32_t lane32 = 4u * (uint32_t)(tid & 31);  // the lane's replica byte offset
  // the nibble tables serve ragged segments only: a buffer's first and last
  // (and batch pieces); whole-segment workgroups start streaming at once
  const bool need_T = jobs != nullptr || blockIdx.x == 0 || blockIdx.x == (unsigned)((nseg - 1) % gridDim.x);
  if (DO_CRC && tid < 32) x2n[tid] = x2n_g[tid];
  if (DO_CRC && need_T) {
    // all loads in flight before the LDS stores (one call's latency matters
    // for small inputs)
    uint32_t tv[256 * 32 / CK_THREADS];
#pragma unroll
    for (int k = 0; k < 256 * 32 / CK_THREADS; ++k) tv[k] = nib_g[nib_index(tid + k * CK_THREADS)];
#pragma unroll
    for (int k = 0; k < 256 * 32 / CK_THREADS; ++k) T[tid + k * CK_THREADS] = tv[k];
  }
  __syncthreads();

  uint32_t wg_crc = 0;  // thread 0: this workgroup's merged segments (fin.acc)
  uint64_t wg_s1 = 0, wg_s2 = 0;
  for (size_t seg = blockIdx.x; seg < nseg; seg += gridDim.x) {
    // one buffer, or (batch) segment k of buffer `jobs[seg]` (16-byte aligned)
    const uint8_t *frame = frame0;
    size_t lo = lo0, hi = hi0, kseg = seg;
    if (jobs) {
      const CkJob j = jobs[seg];
      frame = frame0 + j.off;
      lo = 0;
      hi = j.len;
      kseg = j.k;
    }
    const size_t seg_lo = kseg * CK_SEG;
    const size_t s_lo = seg_lo + (size_t)tid * CK_SLICE;
    const size_t v_lo = s_lo > lo ? s_lo : lo;                              // valid start
    const size_t v_hi = (s_lo + CK_SLICE) < hi ? (s_lo + CK_SLICE) : hi;    // valid end
    uint32_t c = 0, s1 = 0, s2 = 0, len = 0;
    const bool whole = seg_lo >= lo && seg_lo + CK_SEG <= hi;
    uint64_t a1 = 0, a2 = 0;  // Adler sums of this thread's bytes, positions weighted to the segment end
    if (whole) {
      // wave w's bytes in rows of 8 KiB; lane l's 16-byte piece q of row r
      // at 8192 r + 1024 q + 16 l: stream j = 4 q + w of the lane is word w
      // of piece q of every row (bit-sliced CRC, see the header)
      const int wv = tid >> 6, ln = tid & 63;
      const uint4 *p = reinterpret_cast<const uint4 *>(frame + seg_lo + (size_t)wv * CK_WAVE_BYTES) + ln;
      constexpr int RQ = CK_ROW / 16;  // uint4 per row
      uint32_t P[32];
#pragma unroll
      for (int b = 0; b < 32; ++b) P[b] = 0;
      uint32_t S = 0, KS = 0, QS = 0, W = 0;
      uint4 v[8], nx[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) v[q] = ld_stream(p + q * 64);
      // one row: Adler sums of its 8 pieces, the CRC streams one row on
      auto row = [&](const uint4 (&x8)[8], int r, const uint32_t (&pin)[32], uint32_t (&pout)[32]) {
        if (DO_ADLER) {
#pragma unroll
          for (int q = 0; q < 8; ++q) {
            const uint4 x = x8[q];
            uint32_t wsum = __builtin_amdgcn_udot4(x.x, 0x0D0E0F10u, 0u, false);
            wsum = __builtin_amdgcn_udot4(x.y, 0x090A0B0Cu, wsum, false);
            wsum = __builtin_amdgcn_udot4(x.z, 0x05060708u, wsum, false);
            wsum = __builtin_amdgcn_udot4(x.w, 0x01020304u, wsum, false);
            uint32_t sk = __builtin_amdgcn_udot4(x.x, 0x01010101u, 0u, false);
            sk = __builtin_amdgcn_udot4(x.y, 0x01010101u, sk, false);
            sk = __builtin_amdgcn_udot4(x.z, 0x01010101u, sk, false);
            sk = __builtin_amdgcn_udot4(x.w, 0x01010101u, sk, false);
            S += sk;
            KS += (uint32_t)r * sk;
            QS += (uint32_t)q * sk;
            W += wsum;
          }
        }
        if (DO_CRC) {
          uint32_t d[32];
#pragma unroll
          for (int q = 0; q < 8; ++q) {
            d[4 * q] = x8[q].x;
            d[4 * q + 1] = x8[q].y;
            d[4 * q + 2] = x8[q].z;
            d[4 * q + 3] = x8[q].w;
          }
          transpose32(d);
          gf_mul_planes<cx_x8n(CK_ROW)>(pin, d, pout);  // every stream: one row on
        }
      };
      static_assert(CK_ROWS % 2 == 0, "rows go in pairs");
      uint32_t Q[32];
#if ZT_CK_DEPTH == 3
      // three rows in registers: row r + 2's loads are issued while row r is
      // processed (CRC planes ping-pong P / Q by row parity)
      static_assert(CK_ROWS % 6 == 2 && CK_ROWS >= 8, "the 6-row rotation ends on 2 rows in v / nx");
      uint4 w3[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) nx[q] = ld_stream(p + RQ + q * 64);
      auto ld_row = [&](uint4 (&x8)[8], int r) {
#pragma unroll
        for (int q = 0; q < 8; ++q) x8[q] = ld_stream(p + r * RQ + q * 64);
      };
#pragma unroll 1
      for (int r = 0; r + 8 <= CK_ROWS; r += 6) {
        ld_row(w3, r + 2);
        row(v, r, P, Q);
        ld_row(v, r + 3);
        row(nx, r + 1, Q, P);
        ld_row(nx, r + 4);
        row(w3, r + 2, P, Q);
        ld_row(w3, r + 5);
        row(v, r + 3, Q, P);
        ld_row(v, r + 6);
        row(nx, r + 4, P, Q);
        ld_row(nx, r + 7);
        row(w3, r + 5, Q, P);
      }
      row(v, CK_ROWS - 2, P, Q);
      row(nx, CK_ROWS - 1, Q, P);
#else
#pragma unroll 1
      for (int r = 0; r < CK_ROWS; r += 2) {
        // rows r (v) and r + 1 (nx): registers ping-pong, no copies
#pragma unroll
        for (int q = 0; q < 8; ++q) nx[q] = ld_stream(p + (r + 1) * RQ + q * 64);
        row(v, r, P, Q);
        if (r + 2 < CK_ROWS) {
#pragma unroll
          for (int q = 0; q < 8; ++q) v[q] = ld_stream(p + (r + 2) * RQ + q * 64);
        }
        row(nx, r + 1, Q, P);
      }
#endif
      if (DO_CRC) {
        // (the planes are pinned here: LLVM otherwise moves the folds below
        // into the row loop and runs them, selected away, on every row)
#pragma unroll
        for (int b = 0; b < 32; ++b) asm volatile("" : "+v"(P[b]));
        // fold the streams: j and j + h, whose words are D_h bytes apart, into j
        uint32_t t[32], u[32];
#define CK_FOLD(H, D)                                                   \
  {                                                                     \
    _Pragma("unroll") for (int b = 0; b < 32; ++b) t[b] = P[b] >> (H);  \
    gf_mul_planes<cx_x8n(D)>(P, t, u);                                  \
    _Pragma("unroll") for (int b = 0; b < 32; ++b) P[b] = u[b];         \
  }
        CK_FOLD(16, 4096)
        CK_FOLD(8, 2048)
        CK_FOLD(4, 1024)
        CK_FOLD(2, 8)
        CK_FOLD(1, 4)
#undef CK_FOLD
        uint32_t y = 0;
#pragma unroll
        for (int b = 0; b < 32; ++b) y |= (P[b] & 1u) << b;
        c = y;  // the lane's register before its last word's 32 bit steps (folded into its shift)
      }
      len = CK_SLICE;
      // byte k of piece q of row r sits CK_SEG - (wave_off + 8192 r + 1024 q + 16 l + k) bytes before the segment end
      const uint64_t cw = (uint64_t)CK_SEG - (uint64_t)wv * CK_WAVE_BYTES - 16ull * (uint32_t)ln - 16u;
      a1 = S;
      a2 = cw * S - (uint64_t)CK_ROW * KS - 1024ull * QS + W;
    } else if (v_lo == s_lo && v_hi == s_lo + CK_SLICE) {
      len = CK_SLICE;
      const uint4 *p = reinterpret_cast<const uint4 *>(frame + s_lo);
#pragma unroll 1
      for (int line = 0; line < CK_SLICE / 128; ++line) {
        uint4 v[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = ld_stream(p + line * 8 + k);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          if (DO_CRC) {
            c = crc_step8(c, v[k].x, v[k].y, T, lane32);
            c = crc_step8(c, v[k].z, v[k].w, T, lane32);
          }
          if (DO_ADLER) adler16(s1, s2, v[k]);
        }
      }
    } else if (v_lo < v_hi) {
      // ragged slice (first/last segment only): byte at a time
      len = (uint32_t)(v_hi - v_lo);
      size_t i = v_lo;
      if (DO_CRC) {
        // 8 bytes per step through the nibble tables, the rest a byte at a time
        for (; i + 8 <= v_hi; i += 8) {
          uint32_t w0 = 0, w1 = 0;
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            w0 |= (uint32_t)frame[i + k] << (8 * k);
            w1 |= (uint32_t)frame[i + 4 + k] << (8 * k);
          }
          c = crc_step8(c, w0, w1, T, lane32);
        }
        for (; i < v_hi; ++i) c = crc_byte(c, frame[i]);
      }
      if (DO_ADLER) {
        for (size_t j = v_lo; j < v_hi; ++j) {
          s1 += frame[j];
          s2 += s1;
        }
      }
    }
    // ---- merge slices inside the segment ----
    if (DO_ADLER) {
      if (!whole) {
        // bytes after this slice within the segment's valid range
        const size_t seg_v_hi = (seg_lo + CK_SEG) < hi ? (seg_lo + CK_SEG) : hi;
        const size_t after = (v_hi >= v_lo && seg_v_hi > v_hi) ? seg_v_hi - (v_hi > v_lo ? v_hi : v_lo) : 0;
        a1 = s1;
        a2 = (uint64_t)s2 + (uint64_t)s1 * (len ? after : 0);
      }
      for (int off = 32; off > 0; off >>= 1) {
        a1 += __shfl_down(a1, off, 64);
        a2 += __shfl_down(a2, off, 64);
      }
      if ((tid & 63) == 0) {
        red_a[tid >> 6][0] = a1;
        red_a[tid >> 6][1] = a2;
      }
    }
    // a whole segment: thread t's lane stream moves to the segment end (one
    // multiplication by its fixed shift); a ragged one: slice t's CRC over the
    // bytes after it (digit-table shifts); then XOR
    if (DO_CRC) {
      uint32_t x;
      if (whole) {
        x = multmodp(shift_g[ZT_CRC_LANE_OFF + tid], c);
      } else {
        const size_t seg_v_hi = (seg_lo + CK_SEG) < hi ? (seg_lo + CK_SEG) : hi;
        const uint64_t after = (len && seg_v_hi > v_hi) ? seg_v_hi - v_hi : 0;
        x = len ? shift_bytes(shift_g + ZT_CRC_DIG_OFF, x2n, after, c) : 0u;
      }
      for (int off = 32; off > 0; off >>= 1) x ^= (uint32_t)__shfl_xor((int)x, off, 64);
      if ((tid & 63) == 0) red_w[tid >> 6] = x;
    }
    __syncthreads();
    if (DO_CRC && tid == 0) {
      uint32_t x = 0;
      for (int w = 0; w < CK_THREADS / 64; ++w) x ^= red_w[w];
      red_c[0] = x;
    }
    __syncthreads();
    if (tid < 64) {
      // move the segment over the bytes that follow it in the buffer so the
      // finish is a plain XOR / sum: x^(8 * after) as the product of the
      // base-64 digit factors, one per lane 0..7, by a 3-level butterfly
      const size_t sv_lo = seg_lo > lo ? seg_lo : lo;
      const size_t sv_hi = (seg_lo + CK_SEG) < hi ? (seg_lo + CK_SEG) : hi;
      const uint64_t after = hi - sv_hi;
      uint32_t f = 1u << 31;  // x^0
      if (DO_CRC) {
        if (tid < ZT_CRC_DIGITS) {
          const uint32_t v = (uint32_t)(after >> (6 * tid)) & 63u;
          if (v) f = shift_g[ZT_CRC_DIG_OFF + tid * 64 + v];
        }
        for (int o = 1; o < 8; o <<= 1) f = multmodp(f, (uint32_t)__shfl_xor((int)f, o, 64));
      }
      if (tid == 0) {
        SegResult r;
        r.crc = 0;
        if (DO_CRC) {
          uint32_t x = multmodp(f, red_c[0]);
          const uint64_t rest = after >> (6 * ZT_CRC_DIGITS);
          if (rest) x = multmodp(x2nmodp(x2n, rest, 3 + 6 * ZT_CRC_DIGITS), x);
          r.crc = x;
        }
        uint64_t t1 = 0, t2 = 0;
        if (DO_ADLER) {
          for (int w = 0; w < CK_THREADS / 64; ++w) {
            t1 += red_a[w][0];
            t2 += red_a[w][1];
          }
        }
        r.s1 = (uint32_t)(t1 % 65521u);
        r.s2 = (uint32_t)((t2 % 65521u + (after % 65521u) * r.s1) % 65521u);
        r.len = sv_hi > sv_lo ? (uint32_t)(sv_hi - sv_lo) : 0;
        if (fin.acc) {
          wg_crc ^= r.crc;
          wg_s1 += r.s1;
          wg_s2 += r.s2;
        } else {
          out[seg] = r;
        }
      }
    }
    __syncthreads();
  }
  if (fin.acc) {
    // CRC32.update: ~(shift(~crc_in, n) ^ raw); Adler32.update below
    if (DO_CRC && blockIdx.x == 0 && tid == 0) wg_crc ^= shift_bytes(shift_g + ZT_CRC_DIG_OFF, x2n, fin.n, ~fin.crc_in);
    // Device-scope atomics are performed past the XCD's L2, and a returned
    // value means this one has been: a workgroup's partial sums go to its own
    // slot by exchanges, and its ticket is taken only after they returned (no
    // __threadfence: an L2 write-back + invalidate per workgroup, which made
    // the kernel 0.223 -> 0.258 ms).  Tickets: one per group of workgroups
    // (128 bytes apart), the group's last takes the top one -- one counter for
    // every workgroup serialised ~1 K same-address atomics at the kernel's end
    CkAcc *a = fin.acc;
    __shared__ uint32_t s_last;
    if (tid == 0) {
      CkPart *pp = &a->part[blockIdx.x];
      uint32_t landed = atomicExch(&pp->crc, wg_crc);
      landed ^= (uint32_t)atomicExch(&pp->s1, (unsigned long long)wg_s1);
      landed ^= (uint32_t)atomicExch(&pp->s2, (unsigned long long)wg_s2);
      asm volatile("" ::"v"(landed) : "memory");  // waits for the returns
      const uint32_t G = gridDim.x < (uint32_t)kCkGroups ? gridDim.x : (uint32_t)kCkGroups;
      const uint32_t g = blockIdx.x % G;
      const uint32_t members = (gridDim.x - g + G - 1) / G;
      uint32_t last = 0;
      if (atomicAdd(&a->grp[g * 32], 1u) == members - 1) {
        atomicExch(&a->grp[g * 32], 0u);
        last = atomicAdd(&a->done, 1u) == G - 1 ? 1u : 0u;
      }
      s_last = last;
    }
    __syncthreads();
    if (s_last) {
      // (read-modify-writes: the values at the point where the atomics landed)
      uint32_t raw = 0;
      unsigned long long r1 = 0, r2 = 0;
      for (uint32_t w = tid; w < gridDim.x; w += CK_THREADS) {
        CkPart *pp = &a->part[w];
        raw ^= atomicOr(&pp->crc, 0u);
        r1 += atomicAdd(&pp->s1, 0ull) % 65521u;
        r2 += atomicAdd(&pp->s2, 0ull) % 65521u;
      }
      for (int off = 32; off > 0; off >>= 1) {
        raw ^= (uint32_t)__shfl_xor((int)raw, off, 64);
        r1 += __shfl_xor(r1, off, 64);
        r2 += __shfl_xor(r2, off, 64);
      }
      if ((tid & 63) == 0) {
        red_w[tid >> 6] = raw;
        red_a[tid >> 6][0] = r1;
        red_a[tid >> 6][1] = r2;
      }
      __syncthreads();
      if (tid == 0) {
        raw = 0;
        r1 = r2 = 0;
        for (int w = 0; w < CK_THREADS / 64; ++w) {
          raw ^= red_w[w];
          r1 += red_a[w][0];
          r2 += red_a[w][1];
        }
        r1 %= 65521u;
        r2 %= 65521u;
        atomicExch(&a->done, 0u);
        fin.result[0] = ~raw;
        // s1 = adler & 0xFFFF, s2 = (adler >> 16) & 0xFFFF (need not be reduced)
        const uint64_t a1 = fin.adler_in & 0xFFFFu, a2 = (fin.adler_in >> 16) & 0xFFFFu;
        const uint64_t f1 = (a1 + r1) % 65521u;
        const uint64_t f2 = (a2 + (fin.n % 65521u) * (a1 % 65521u) + r2) % 65521u;
        fin.result[1] = (uint32_t)((f2 << 16) | f1);
      }
    }
  }
}

// batch: one lane per buffer, its segments [first[i], first[i + 1]) merged
__global__ __launch_bounds__(256) void checksum_batch_finish(const SegResult *__restrict__ segs,
                                                             const uint32_t *__restrict__ first,
                                                             const uint64_t *__restrict__ lens, uint32_t count,
                                                             const uint32_t *__restrict__ x2n_g,
                                                             const uint32_t *__restrict__ shift_g,
                                                             uint32_t *__restrict__ result) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i >= count) return;
  uint32_t raw = 0;
  uint64_t t1 = 0, t2 = 0;
  for (uint32_t k = first[i]; k < first[i + 1]; ++k) {
    const SegResult r = segs[k];
    raw ^= r.crc;
    t1 += r.s1;
    t2 += r.s2;
  }
  const uint64_t n = lens[i];
  result[2 * i] = ~(shift_bytes(shift_g + ZT_CRC_DIG_OFF, x2n_g, n, 0xFFFFFFFFu) ^ raw);
  const uint64_t f1 = (1 + t1 % 65521u) % 65521u;
  const uint64_t f2 = ((n % 65521u) + t2 % 65521u) % 65521u;
  result[2 * i + 1] = (uint32_t)((f2 << 16) | f1);
}

}  // namespace

void crc_host_tables(uint32_t byte_table[256], uint32_t nib[ZT_CRC_NIB_N], uint32_t x2n[32]) {
  for (uint32_t i = 0; i < 256; ++i) {
    uint32_t c = i;
    for (int j = 0; j < 8; ++j) c = (c & 1) ? (ZT_CRC_POLY ^ (c >> 1)) : (c >> 1);
    byte_table[i] = c;
  }
  // nib[pos*16 + v]: raw CRC (init 0) of an 8-byte block whose only non-zero
  // nibble is v at nibble position pos (byte pos/2, high half when pos is odd)
  for (int pos = 0; pos < 16; ++pos) {
    for (uint32_t v = 0; v < 16; ++v) {
      uint8_t blk[8] = {0};
      blk[pos >> 1] = (uint8_t)(v << (4 * (pos & 1)));
      uint32_t c = 0;
      for (int k = 0; k < 8; ++k) c = (c >> 8) ^ byte_table[(c ^ blk[k]) & 0xFF];
      nib[pos * 16 + v] = c;
    }
  }
  x2n[0] = 1u << 30;  // x^1
  for (int k = 1; k < 32; ++k) x2n[k] = multmodp(x2n[k - 1], x2n[k - 1]);
  // (entries [256, 384) unused: the whole-segment path is table-free)
  for (int i = 256; i < ZT_CRC_NIB_N; ++i) nib[i] = 0;
}

void crc_shift_tables(const uint32_t x2n[32], uint32_t shift[ZT_CRC_SHIFT_N]) {
  // lanes of a whole segment: thread t = 64 w + l holds y with its CRC
  // register = y * x^32, ending CK_WAVE_BYTES (waves - 1 - w) + 1024 - 16 (l +
  // 1) bytes before the segment end (bit-sliced path, checksum_segments):
  // the shift x^(8 after + 32)
  for (int t = 0; t < CK_THREADS; ++t) {
    const uint64_t after =
        (uint64_t)CK_WAVE_BYTES * (CK_THREADS / 64 - 1 - t / 64) + 1024 - 16 * (uint64_t)(t % 64 + 1);
    shift[ZT_CRC_LANE_OFF + t] = x2nmodp(x2n, after + 4, 3);
  }
  // digit tables: x^(8 * v * 64^d)
  for (int d = 0; d < ZT_CRC_DIGITS; ++d)
    for (uint64_t v = 0; v < 64; ++v) shift[ZT_CRC_DIG_OFF + d * 64 + v] = x2nmodp(x2n, v << (6 * d), 3);
}

// CRC-32 and Adler-32 (initial values 0 and 1) of `count` buffers at
// frame + off[i] (16-byte aligned) in one launch pair: d_result[2 i] = CRC,
// d_result[2 i + 1] = Adler.  Empty buffers give 0 / 1.
int checksums_batch_dev(DeviceCtx *c, const uint8_t *frame, size_t count, const uint64_t *off, const uint64_t *len,
                        uint32_t *d_result, hipStream_t s) {
  if (count == 0) return ZT_OK;
  std::vector<CkJob> jobs;
  std::vector<uint32_t> first(count + 1);
  for (size_t i = 0; i < count; ++i) {
    if (off[i] & 15) return set_error(ZT_E_ARG, "batch checksum buffers must be 16-byte aligned");
    first[i] = (uint32_t)jobs.size();
    const uint64_t ns = (len[i] + CK_SEG - 1) / CK_SEG;
    for (uint64_t k = 0; k < ns; ++k) jobs.push_back(CkJob{off[i], len[i], k});
  }
  first[count] = (uint32_t)jobs.size();
  const size_t nj = jobs.size();
  const size_t jb = (nj * sizeof(CkJob) + 255) & ~size_t(255), fb = ((count + 1) * 4 + 255) & ~size_t(255);
  const size_t lb = (count * 8 + 255) & ~size_t(255), sb = ((nj ? nj : 1) * sizeof(SegResult) + 255) & ~size_t(255);
  void *buf;
  ZT_TRY(scratch(c, 9, jb + fb + lb + sb, &buf));
  uint8_t *b = static_cast<uint8_t *>(buf);
  CkJob *d_jobs = reinterpret_cast<CkJob *>(b);
  uint32_t *d_first = reinterpret_cast<uint32_t *>(b + jb);
  uint64_t *d_len = reinterpret_cast<uint64_t *>(b + jb + fb);
  SegResult *d_seg = reinterpret_cast<SegResult *>(b + jb + fb + lb);
  // small tables: blocking copies (the kernels below stay asynchronous)
  if (nj) ZT_HIP(hipMemcpy(d_jobs, jobs.data(), nj * sizeof(CkJob), hipMemcpyHostToDevice));
  ZT_HIP(hipMemcpy(d_first, first.data(), (count + 1) * 4, hipMemcpyHostToDevice));
  ZT_HIP(hipMemcpy(d_len, len, count * 8, hipMemcpyHostToDevice));
  if (nj) {
    checksum_segments<true, true><<<(unsigned)nj, CK_THREADS, 0, s>>>(frame, 0, 0, nj, c->d_crc_nib, c->d_crc_x2n,
                                                                      c->d_crc_shift, d_seg, d_jobs, CkFinish{});
    ZT_HIP(hipGetLastError());
  }
  checksum_batch_finish<<<(unsigned)((count + 255) / 256), 256, 0, s>>>(d_seg, d_first, d_len, (uint32_t)count,
                                                                        c->d_crc_x2n, c->d_crc_shift, d_result);
  ZT_HIP(hipGetLastError());
  return ZT_OK;
}

int checksums_dev(DeviceCtx *c, const uint8_t *d_in, size_t n, bool do_crc, bool do_adler, uint32_t crc_in,
                  uint32_t adler_in, uint32_t *d_result, hipStream_t s) {
  const uintptr_t addr = reinterpret_cast<uintptr_t>(d_in);
  const uint8_t *frame = reinterpret_cast<const uint8_t *>(addr & ~uintptr_t(15));
  const size_t lo = addr & 15, hi = lo + n;
  const size_t nseg = n ? (hi + CK_SEG - 1) / CK_SEG : 1;
  void *segbuf;
  ZT_TRY(scratch(c, 8, nseg * sizeof(SegResult), &segbuf));
  SegResult *segs = static_cast<SegResult *>(segbuf);
  size_t g = nseg < (size_t)c->num_cu * 8 ? nseg : (size_t)c->num_cu * 8;
  if (g > (size_t)kCkMaxWg) g = kCkMaxWg;  // (one partial slot per workgroup)
  const int grid = (int)g;
  const CkFinish fin{c->d_ck_acc, d_result, n, crc_in, adler_in};
  if (do_crc && do_adler)
    checksum_segments<true, true><<<grid, CK_THREADS, 0, s>>>(frame, lo, hi, nseg, c->d_crc_nib, c->d_crc_x2n,
                                                              c->d_crc_shift, segs, nullptr, fin);
  else if (do_crc)
    checksum_segments<true, false><<<grid, CK_THREADS, 0, s>>>(frame, lo, hi, nseg, c->d_crc_nib, c->d_crc_x2n,
                                                               c->d_crc_shift, segs, nullptr, fin);
  else
    checksum_segments<false, true><<<grid, CK_THREADS, 0, s>>>(frame, lo, hi, nseg, c->d_crc_nib, c->d_crc_x2n,
                                                               c->d_crc_shift, segs, nullptr, fin);
  ZT_HIP(hipGetLastError());
  return ZT_OK;
}

}  // namespace zt
