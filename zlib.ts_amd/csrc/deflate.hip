// deflate.hip -- raw DEFLATE (RFC 1951) encoder on the GPU.
// Replaces src/LZ77.ts, src/RawDeflate.ts, src/Heap.ts and src/Bitstream.ts.
//
// Kernels over device memory, each shaped for the phase it runs:
//
//   1. match_kernel -- one 1024-thread workgroup per super-chunk (4
//      consecutive 32 KiB blocks; a 1 MiB segment starts without history,
//      later super-chunks index the 28 KiB before them first).  4 KiB
//      sub-chunks stream through a 32 KiB LDS ring (28 608-byte window).
//      Wave 0 links 8-byte-key hash chains (u32 heads, u16 relative links)
//      and wave 1 a 4-byte-key table (the newest earlier position per
//      bucket), each by lane-ordered LDS exchanges head[h] <-> p, 64
//      positions per exchange, publishing their progress; all waves search
//      256-position super-steps as soon as they are linked: per thread 4
//      positions, two chain walks interleaved (two LDS loads per hop: the
//      link and one filter word), candidates measured against 16 bytes held
//      in registers; matches shorter than the key come from near probes
//      (distances 1..16, register window) and the 4-byte table.  The
//      longest match of every position goes to HBM: res[i] = len << 16 |
//      dist.
//   2. price_kernel + optparse_kernel -- one wave per 32 KiB block: bit
//      prices from the greedy parse of the block's first quarter, then a
//      backward shortest-path DP over every position (cut lengths 3..16 and
//      the full match), choices written over res.
//   3. parse_kernel -- one wave per block: parse of the DP's choices
//      (LDS-DMA staged, pointer doubling), tokens over res, histograms (a
//      small LDS footprint: many waves per CU).
//      block_kernel -- one wave per block: length-limited Huffman lengths by
//      wave-parallel package-merge, canonical codes, the RLE'd code-length
//      header, and the smallest of stored / fixed / dynamic.
//   4. encode_kernel -- 512 threads per block: prefix sum of per-thread bit
//      counts, word-parallel packing; every block ends byte-aligned with an
//      empty stored block (00 00 FF FF) so blocks concatenate bytewise.
//   5. scan_sizes (before encode_kernel: block_kernel plans every block's
//      exact size) places each block, encode_kernel writes it there; 1 MiB segment boundaries
//      get a restart marker (two empty stored blocks) for segment-parallel
//      inflate (inflate_seg.hip).
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "zt_internal.h"

namespace zt {

#ifdef ZT_DF_TIME
__device__ unsigned long long g_df_time[8];  // debug: cycles (thread 0 of each workgroup) in phases
__device__ unsigned long long g_bk_time[8];  // debug: block_kernel phase cycles (lane 0), [6] = blocks
#define DF_T(v) v = __builtin_readcyclecounter()
#else
#define DF_T(v) (void)0
#endif
#ifdef ZT_DF_COUNT
__device__ unsigned long long g_df_count[8];  // debug: pair steps (per wave), lane hops, extends (lanes), extends (waves),
                                              // measured lanes that improve / measure < 8 bytes / do not improve
#endif

#ifndef ZT_DF_BLOCK
#define ZT_DF_BLOCK 32768
#endif
constexpr int DF_BLOCK = ZT_DF_BLOCK;
// DEFLATE blocks (one Huffman code, one header, one sync point) may span
// DF_GROUP consecutive 32 KiB parse blocks of a stream (compile option): the
// match / price / DP / parse kernels keep their 32 KiB granularity,
// block_kernel sums the group's histograms and encode_kernel writes the
// group's tokens as one block.  Inflate units are one DEFLATE block
// (inflate_seg.hip).  Measured at 4 (profiles/r03b_*): wordsalad ratio vs the
// reference 1.0168 -> 1.0145 only, but inflate 10.9 -> 12.2 ms per GiB
// (tokenize and expand get a quarter of the units): kept at 1.
#ifndef ZT_DF_GROUP
#define ZT_DF_GROUP 1
#endif
constexpr int DF_GROUP = ZT_DF_GROUP;
static_assert(DF_GROUP >= 1 && DF_GROUP <= 8 && (32 % DF_GROUP) == 0, "group divides a segment");
constexpr int DF_SUB = 4096;
constexpr int DF_RING = 32768;  // power of two: ring index = rel & (DF_RING - 1)
// per-block slot: the block's prices (price_kernel -> optparse_kernel), then
// its histograms and token count (parse_kernel -> block_kernel), then its
// dynamic header's complete words (block_kernel -> encode_kernel: at most
// 17 + 19 * 3 + 316 * 14 bits); the coded block itself goes straight into the stream
constexpr int DF_SLOT = 2048;
static_assert(DF_SLOT >= 321 * 4 && DF_SLOT * 8 >= 17 + 19 * 3 + 316 * 14, "slot holds histograms and a header");
// hash buckets of the 8-byte-key chains (u32 heads) and of the 4-byte-key
// table (u32 heads, no chains): the sizes fill the 160 KiB of LDS next to the
// ring, the chain links and the sub-chunk's 4-byte links
#ifndef ZT_DF_HSIZE
#ifdef ZT_DF_HEAD16
#define ZT_DF_HSIZE 24528  // (u16 heads, two per word)
#else
#define ZT_DF_HSIZE 12240
#endif
#endif
#ifndef ZT_DF_H4SIZE
#define ZT_DF_H4SIZE 2048
#endif
#ifndef ZT_DF_P4FAR
#define ZT_DF_P4FAR 1024  // 4-byte (not longer) matches from the 4-byte-key table reach at most this far
#endif
constexpr uint32_t DF_HSIZE = ZT_DF_HSIZE;
constexpr uint32_t DF_H4SIZE = ZT_DF_H4SIZE;
static_assert(DF_HSIZE <= 65536 && DF_H4SIZE <= 65536, "bucket indices are parked in u16 slots (hash_keys)");
constexpr int DF_THREADS = 1024;
// the ring holds [p1 - DF_RING, p1) while sub-chunk [p0, p1) is searched;
// a super-chunk loads DF_HIST bytes of history first (whole sub-chunks)
constexpr int DF_HIST = DF_RING - DF_SUB;     // 28672
// The first DF_HEAD bytes of the next sub-chunk are in the ring while a
// sub-chunk is searched, so matches run on past its end (to the block's);
// they take the ring slots of the window's oldest DF_HEAD - 64 bytes.
#ifndef ZT_DF_HEAD
#define ZT_DF_HEAD 320
#endif
constexpr int DF_HEAD = ZT_DF_HEAD;
static_assert(DF_HEAD == 0 || DF_HEAD >= 258 + 8 + 54, "a head covers a whole match past the sub-chunk end");
constexpr int DF_MAXDIST = DF_HIST - 64 - (DF_HEAD ? DF_HEAD - 64 : 0);  // 28352 (28608 without heads)
#ifndef ZT_ENC_THREADS
#define ZT_ENC_THREADS 512  // 128 / 256 / 512 / 1024: 1.70 / 1.42 / 1.38 / 1.75 ms per GiB (profiles/r02q_encode_variants.txt)
#endif
constexpr int ENC_THREADS = ZT_ENC_THREADS;
// Independent segments of 1 MiB: restart points for segment-parallel inflate
constexpr uint32_t kRestartBlocks = (1u << 20) / DF_BLOCK;  // 1 MiB
// empty head entry: p - kNoHead exceeds DF_MAXDIST for every rel position p
constexpr uint32_t kNoHead = 0x80000000u;

struct BlockPlan;

struct DeflateParams {
  const uint8_t *base;  // stream bytes are base[halo .. halo + n)
  uint64_t halo;
  uint64_t end;         // halo + n
  uint32_t blocks_per_wg;
  uint32_t big_wgs;     // match workgroups [0, big_wgs) take blocks_per_wg blocks, later ones tail_k
  uint32_t tail_k;
  uint32_t nblocks;
  uint32_t restart;     // blocks per independent segment (multiple of blocks_per_wg)
  uint32_t hist_max;    // history bytes a super-chunk loads (multiple of DF_SUB, <= DF_HIST)
  int final_;
  int max_chain;
  int nice_len;
  int lazy;
  int too_far;
  int good;             // a carried match this long cuts the chain walk to a quarter
  int skip_len;         // a carried match at least this long is taken without a search
  int klen;             // chain key length: 3, 4, 6 or 8 bytes (shorter matches come from near probes)
  int probe;            // near distances 1..probe checked for matches shorter than klen
  int ctype;            // 1: fixed codes only; 2: best of dynamic/fixed/stored
  int opt;              // cost-based parse (optparse_kernel) between match and block kernels
  // Per-block search depth (0: off): the block's first sub-chunk is searched
  // with max_chain hops and counts the improvements its walks found at hop
  // adapt_depth or later (and at hop adapt_depth2 or later); when the first
  // are at most adapt_thr per 4096 positions, the rest of the block walks
  // adapt_depth hops, else when the second are at most adapt_thr2,
  // adapt_depth2 hops (match_kernel)
  int adapt_depth, adapt_thr;
  int adapt_depth2, adapt_thr2;
  // batch of independent streams (zt_deflate_batch_dev): stream f occupies
  // whole blocks from a 32 KiB-aligned offset; per block the [start, end) of
  // its stream (relative to halo = 0), or null for one stream of n bytes
  const uint64_t *span;
  // per block: 1 = no match search, a stored block (classify_kernel: bytes
  // that cannot beat stored); null when not classified
  uint8_t *store;
  uint32_t *nstore;     // blocks flagged (one counter, zeroed before classify_kernel)
  uint32_t *res;        // n: per-position match, then (in place) per-block tokens
  uint8_t *slots;       // nblocks x DF_SLOT (prices, histograms, dynamic headers)
  uint32_t *slot_len;   // nblocks: each block's bytes (block_kernel's plan, exact)
  uint8_t *out;         // the stream: encode_kernel writes block b at out + boff[b]
  const uint64_t *boff; // exclusive scan of slot_len (+ restart markers), scan_sizes
  uint32_t *fault;      // encode_kernel: a block's bits differ from its plan
  BlockPlan *plans;     // nblocks
};

// per-block coding decisions (block_kernel -> encode_kernel)
struct BlockPlan {
  uint32_t lit_code[288];  // len << 16 | bit-reversed code
  uint32_t dist_code[32];
  uint32_t ntok;      // tokens of the group
  uint32_t btype;     // 0 stored, 1 fixed, 2 dynamic
  uint32_t hdr_bits;  // header bits (complete words already in the slot)
  uint32_t hdr_tail;  // bits [hdr_bits & ~31, hdr_bits) of the header, not yet stored
  uint32_t blen;      // input bytes of the group
  uint32_t last;
  uint32_t nsub;      // parse blocks in the group (<= DF_GROUP)
  uint32_t pad;
  uint32_t ntok_sub[8];  // tokens per parse block (in res at (leader + k) * DF_BLOCK)
};

namespace {

// end of the stream block `blk` belongs to (relative to base + halo)
__device__ __forceinline__ uint64_t stream_end(const DeflateParams &P, uint32_t blk) {
  return P.span ? P.span[2 * (uint64_t)blk + 1] : P.end - P.halo;
}

// a DEFLATE block (group) starts at every DF_GROUP-th parse block of its
// stream (batch: counted from the stream's first block)
__device__ __forceinline__ bool group_leader(const DeflateParams &P, uint32_t blk) {
  const uint64_t first = P.span ? P.span[2 * (uint64_t)blk] / DF_BLOCK : 0;
  return ((blk - first) % DF_GROUP) == 0;
}
// parse blocks in the group led by `blk`
__device__ __forceinline__ uint32_t group_size(const DeflateParams &P, uint32_t blk) {
  const uint64_t lo = (uint64_t)blk * DF_BLOCK, n = stream_end(P, blk);
  const uint64_t nb = (n - lo + DF_BLOCK - 1) / DF_BLOCK;
  return nb < (uint64_t)DF_GROUP ? (uint32_t)nb : (uint32_t)DF_GROUP;
}

__constant__ uint8_t kClOrder[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

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

__device__ __forceinline__ uint32_t len_sym(uint32_t L) {  // 0..28 (symbol - 257)
  if (L == 258) return 28;
  if (L <= 10) return L - 3;
  uint32_t x = L - 3;
  uint32_t k = 31 - __clz(x);  // >= 3
  return 4 * (k - 1) + ((x >> (k - 2)) & 3);
}

// Per-position match word in res (match_kernel -> price / optparse / parse):
// the byte at the position in bits 24-31 (so the later kernels never read
// the input again), the match length (0 or 3..258) in bits 15-23 and its
// distance (<= DF_MAXDIST < 2^15) in bits 0-14.  optparse_kernel rewrites the
// length with its choice (0 = literal).
__device__ __forceinline__ uint32_t res_pack(uint32_t byte, uint32_t len, uint32_t dist) {
  return (byte << 24) | (len << 15) | dist;
}
__device__ __forceinline__ uint32_t res_len(uint32_t r) { return (r >> 15) & 511u; }
__device__ __forceinline__ uint32_t res_dist(uint32_t r) { return r & 0x7FFFu; }
__device__ __forceinline__ uint32_t res_byte(uint32_t r) { return r >> 24; }

// ================================ 0. classify_kernel ================================
// Blocks that cannot beat a stored block skip the match search and the parse
// (src/RawDeflate.ts:122-153 is the stored form).  Decided
// from the block's bytes alone, one 256-thread workgroup per 32 KiB block:
//  A. order-0 entropy of a 4 KiB sample (1 KiB at each quarter): below
//     CL_ENTROPY bits per byte the literals alone would compress -> search;
//  B. high-entropy blocks are checked for repeats (random data that occurs
//     twice compresses although its bytes look random): the 8-byte keys of
//     every 16th position of the window (up to 28 KiB of history in the same
//     segment + the block) go into an LDS table (position + a 16-bit
//     fingerprint per bucket), every position of the block looks its key up
//     from registers (each thread 128 consecutive positions); a repeat of L
//     bytes gives ~L / 16 hits (the pair's other position, before or after,
//     within a match distance).  CL_HITS hits or more -> search.
//  C. the block's byte histogram (every 3rd byte, from the registers stage B
//     loaded): a block whose order-0 entropy would let an ideal literal coder
//     save more than CL_SAVE over the stored form is searched (a skewed
//     block -- 7.85..7.98 bits -- or compressible bytes outside the sample).
// Everything else is flagged: match / price / DP / parse skip the block and
// block_kernel plans it stored (the smallest form for such bytes: the
// reference's dynamic block of random data is 0.1 % larger).
constexpr float CL_ENTROPY = 7.85f;  // uniform bytes: ~7.955 from a 4096-byte sample
constexpr uint32_t CL_HITS = 8;
constexpr float CL_SAVE = 0.002f;  // C: largest saving an ideal literal coder may forgo
constexpr int CL_STRIDE = 3;       // C: every 3rd byte counted
constexpr uint32_t CL_TABLE = 8192;
constexpr uint32_t CL_EMPTY = 0xFFFFFFFFu;
struct ClassifyShared {
  uint32_t table[CL_TABLE];  // window position << 16 | fingerprint
  uint32_t hist[256];
  float part[4];
  uint32_t hits[4];
  float cnt[4][2];  // stage C: bytes counted, bins used (per wave)
};

// 4 stream bytes at g + off (off >= 0 relative to a possibly unaligned g);
// bytes at or past `end` read as 0
__device__ __forceinline__ uint32_t cl_gword(const uint8_t *g, int64_t off, uint64_t end) {
  const uint8_t *a = g + off;
  if ((reinterpret_cast<uintptr_t>(a) & 3) == 0 && off + 4 <= (int64_t)end)
    return *reinterpret_cast<const uint32_t *>(a);
  uint32_t v = 0;
  for (int k = 0; k < 4; ++k)
    if (off + k < (int64_t)end) v |= (uint32_t)a[k] << (8 * k);
  return v;
}
// 13-bit bucket and 16-bit fingerprint of an 8-byte key
__device__ __forceinline__ uint32_t cl_hash(uint32_t a, uint32_t b) {
  uint32_t h = a * 0x9E3779B1u ^ b * 0x85EBCA77u;
  h ^= h >> 15;
  return h * 0x2C1B3C6Du;
}

__global__ __launch_bounds__(256) void classify_kernel(DeflateParams P) {
  __shared__ ClassifyShared sh;
  ClassifyShared *s = &sh;
  const uint32_t t = threadIdx.x, blk = blockIdx.x;
  const uint64_t lo = (uint64_t)blk * DF_BLOCK;
  const uint64_t n = stream_end(P, blk);
  const uint32_t blen = (uint32_t)((n - lo) < DF_BLOCK ? (n - lo) : DF_BLOCK);
  const uint8_t *g = P.base + P.halo;  // stream byte 0
  if (blen < 4096) {  // (small blocks: a search is cheap)
    if (t == 0) P.store[blk] = 0;
    return;
  }
  // A. entropy of the sample (4 words every `stride` bytes)
  s->hist[t] = 0;
  __syncthreads();
  // (four contiguous 1 KiB pieces, a quarter of the block apart: coalesced,
  // 4 KiB of lines per block instead of one line per sampled word)
  const uint32_t pstep = (blen / 4) & ~15u;
  {
    uint32_t v[4];
    const uint64_t a = lo + (uint64_t)(t >> 6) * pstep + (t & 63) * 16;
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = cl_gword(g, (int64_t)(a + 4 * j), n);
#pragma unroll
    for (int j = 0; j < 16; ++j) atomicAdd(&s->hist[(v[j >> 2] >> (8 * (j & 3))) & 0xFF], 1u);
  }
  __syncthreads();
  const float c = (float)s->hist[t];
  float e = c > 0.f ? c * __log2f(c) : 0.f;
  for (int off = 32; off; off >>= 1) e += __shfl_xor(e, off, 64);
  if ((t & 63) == 0) s->part[t >> 6] = e;
  __syncthreads();
  const float h = 12.0f - (s->part[0] + s->part[1] + s->part[2] + s->part[3]) * (1.0f / 4096.0f);
  if (h < CL_ENTROPY) {
    if (t == 0) P.store[blk] = 0;
    return;
  }
#ifdef ZT_CL_NOB  // (measurement: stage A alone)
  if (t == 0) {
    P.store[blk] = 1;
    atomicAdd(P.nstore, 1u);
  }
  return;
#endif
  // B. repeats inside the window: history from the block's segment / stream
  const uint64_t f_lo = P.span ? P.span[2 * (uint64_t)blk] : 0;
  const uint64_t seg = ((lo - f_lo) / DF_BLOCK) / P.restart;
  const uint64_t w_lo = f_lo + seg * P.restart * DF_BLOCK;  // segment start (stream coordinates)
  const bool halo_hist = !P.span && seg == 0 && P.halo > 0;  // the first segment may look into the halo
  int64_t h0 = (int64_t)lo - DF_HIST;
  const int64_t floor_ = halo_hist ? -(int64_t)(P.halo < (uint64_t)DF_HIST ? P.halo : (uint64_t)DF_HIST) : (int64_t)w_lo;
  if (h0 < floor_) h0 = floor_;
  const uint32_t wlen = (uint32_t)((int64_t)lo + blen - h0);
  for (uint32_t i = t; i < CL_TABLE; i += 256) s->table[i] = CL_EMPTY;
  s->hist[t] = 0;  // (stage A's reads of it are behind the barrier above; B2 counts the whole block)
  // B1. inserts: every 16th position of the window (at most 15 per thread,
  // every load issued before the first is used); 8-byte loads when the
  // stream is 16-byte aligned and the window's reads stay inside it
  constexpr int NI = (DF_HIST + DF_BLOCK) / (16 * 256);
  const bool vec = (reinterpret_cast<uintptr_t>(g) & 15) == 0 && (h0 & 15) == 0 && lo + DF_BLOCK + 8 <= n;
  typedef unsigned int cl_u32x2 __attribute__((ext_vector_type(2)));
  typedef unsigned int cl_u32x4 __attribute__((ext_vector_type(4)));
  {
    uint32_t w[NI][3];
    const int64_t a4 = h0 & ~int64_t(3);
    const uint32_t sh = (uint32_t)(h0 - a4);
    if (vec) {
#pragma unroll
      for (int i = 0; i < NI; ++i) {
        const uint32_t r = 16 * (t + 256 * i);
        const cl_u32x2 v = r + 8 <= wlen ? *reinterpret_cast<const cl_u32x2 *>(g + h0 + r) : cl_u32x2{0, 0};
        w[i][0] = v.x;
        w[i][1] = v.y;
      }
    } else {
#pragma unroll
      for (int i = 0; i < NI; ++i) {
        const int64_t a = a4 + 16 * (int64_t)(t + 256 * i);
#pragma unroll
        for (int j = 0; j < 3; ++j) w[i][j] = cl_gword(g, a + 4 * j, n);
      }
    }
    __syncthreads();  // (the table's EMPTY stores before any insert)
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const uint32_t r = 16 * (t + 256 * i);
      const uint32_t x0 = vec ? w[i][0] : __builtin_amdgcn_alignbyte(w[i][1], w[i][0], sh);
      const uint32_t x1 = vec ? w[i][1] : __builtin_amdgcn_alignbyte(w[i][2], w[i][1], sh);
      const uint32_t hh = cl_hash(x0, x1);
      if (r + 8 <= wlen) s->table[hh >> 19] = (r << 16) | (hh & 0xFFFFu);
    }
  }
  __syncthreads();
  // B2. queries: thread t the 128 positions from lo + 128 t (block coordinates k)
  const uint32_t b0 = (uint32_t)((int64_t)lo - h0);  // the block in window coordinates
  uint32_t hits = 0;
  const uint32_t k0 = 128 * t;
  if (k0 < blen) {
    uint32_t w[36];
    if (vec) {
      const cl_u32x4 *v4 = reinterpret_cast<const cl_u32x4 *>(g + lo + k0);
#pragma unroll
      for (int j = 0; j < 9; ++j) {
        const cl_u32x4 v = v4[j];
        w[4 * j] = v.x;
        w[4 * j + 1] = v.y;
        w[4 * j + 2] = v.z;
        w[4 * j + 3] = v.w;
      }
    } else {
#pragma unroll
      for (int j = 0; j < 34; ++j) w[j] = cl_gword(g, (int64_t)(lo + k0 + 4 * j), n);
    }
    // the block's byte histogram over every 3rd byte (stage A saw a 4 KiB
    // sample only; a stride prime to 2 sees every byte lane of 2-, 4- and
    // 8-byte records; all 32 KiB took 0.23 ms per GiB of LDS atomics)
#pragma unroll
    for (int k = 0; k < 128; k += CL_STRIDE)
      if (k0 + (uint32_t)k < blen) atomicAdd(&s->hist[(w[k >> 2] >> (8 * (k & 3))) & 0xFF], 1u);
#pragma unroll
    for (int k = 0; k < 128; ++k) {
      const uint32_t x0 = (k & 3) ? __builtin_amdgcn_alignbyte(w[(k >> 2) + 1], w[k >> 2], k & 3) : w[k >> 2];
      const uint32_t x1 =
          (k & 3) ? __builtin_amdgcn_alignbyte(w[(k >> 2) + 2], w[(k >> 2) + 1], k & 3) : w[(k >> 2) + 1];
      const uint32_t hh = cl_hash(x0, x1);
      const uint32_t ent = s->table[hh >> 19];
      const uint32_t r = b0 + k0 + (uint32_t)k, q = ent >> 16;
      const bool ok = k0 + (uint32_t)k + 8 <= blen && ent != CL_EMPTY && (ent & 0xFFFFu) == (hh & 0xFFFFu) &&
                      q != r && (q < r ? r - q : q - r) <= (uint32_t)DF_MAXDIST;
      hits += ok ? 1u : 0u;
    }
  }
  for (int off = 32; off; off >>= 1) hits += __shfl_xor(hits, off, 64);
  if ((t & 63) == 0) s->hits[t >> 6] = hits;
  __syncthreads();
  // C. the block's order-0 entropy (Miller-Madow: the sample's plug-in
  // estimate + (bins used - 1) / (2 N ln 2), its bias): an ideal literal
  // coder (which no Huffman code beats) + a 32-byte header must not save more
  // than CL_SAVE of the block over the stored form, or the block is searched
  // (uniform bytes: ~8.00 bits per byte, the cut ~7.98)
  const float cb = (float)s->hist[t];
  float eb = cb > 0.f ? cb * __log2f(cb) : 0.f, nb = cb, kb = cb > 0.f ? 1.f : 0.f;
  for (int off = 32; off; off >>= 1) {
    eb += __shfl_xor(eb, off, 64);
    nb += __shfl_xor(nb, off, 64);
    kb += __shfl_xor(kb, off, 64);
  }
  __syncthreads();  // (every hist read done before part[] is rewritten below)
  if ((t & 63) == 0) {
    s->part[t >> 6] = eb;
    s->cnt[t >> 6][0] = nb;
    s->cnt[t >> 6][1] = kb;
  }
  __syncthreads();
  if (t == 0) {
    const float n = s->cnt[0][0] + s->cnt[1][0] + s->cnt[2][0] + s->cnt[3][0];
    const float k = s->cnt[0][1] + s->cnt[1][1] + s->cnt[2][1] + s->cnt[3][1];
    const float hb = __log2f(n) - (s->part[0] + s->part[1] + s->part[2] + s->part[3]) / n +
                     (k - 1.f) / (2.f * n * 0.69314718f);
    const bool flat = hb * (float)blen * 0.125f + 32.f >= (1.0f - CL_SAVE) * (float)blen;
    const bool st = flat && (s->hits[0] + s->hits[1] + s->hits[2] + s->hits[3]) < CL_HITS;
    P.store[blk] = st ? 1 : 0;
    if (st) atomicAdd(P.nstore, 1u);
  }
}

// ================================ 1. match_kernel ================================
constexpr uint32_t RING_ENT = DF_RING / 4;
struct MatchShared {
  uint32_t ring[DF_RING / 4 + 16];  // data ring + 64-byte mirror of its start
  uint16_t prev[DF_RING];           // relative chain links (0 = none)
#ifdef ZT_DF_HEAD16
  uint32_t head[DF_HSIZE / 2];      // newest position (rel mod 2^16) per hash bucket, two buckets per word
#else
  uint32_t head[DF_HSIZE];          // newest position (rel) per hash bucket
#endif
  uint32_t head4[DF_H4SIZE];        // newest position (rel) per 4-byte-key bucket
  uint16_t link4[DF_SUB];           // position p of the sub-chunk: distance to the newest earlier
                                    // position of its 4-byte-key bucket (0 = none), at p % DF_SUB
  uint32_t dummy[4];                // exchange / link targets of lanes past the end (branch-free chain_link)
  uint32_t linked;                  // positions below are linked (chain_link -> searching waves)
  uint32_t linked4;                 // positions below have their 4-byte links
  uint32_t work;                    // next super-step of 256 positions to search
  uint32_t late, late2;             // probe sub-chunk: improvements at hop >= adapt_depth / adapt_depth2
  int depth;                        // max_chain of the block's later sub-chunks
};

// Workgroup barrier for LDS hand-offs only: waits for this wave's LDS
// operations, not for its global loads (the next sub-chunk's prefetch stays
// in flight) nor its global stores (res[] is read by later kernels only).
// __syncthreads() would drain vmcnt and expose HBM latency at every barrier.
__device__ __forceinline__ void lds_barrier() { __asm__ volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

__device__ __forceinline__ uint32_t ridx(uint32_t rel) { return rel & (DF_RING - 1); }
// ---- ring storage: every access goes through these ----
// dword w (0 <= w < RING_ENT) of the ring := v (and its mirror copies)
__device__ __forceinline__ void ring_put32(MatchShared *s, uint32_t w, uint32_t v) {
  s->ring[w] = v;
  if (w < 16) s->ring[RING_ENT + w] = v;
}
// byte k (0 <= k < DF_RING) of the ring := v (and its copies)
__device__ __forceinline__ void ring_put8(MatchShared *s, uint32_t k, uint8_t v) {
  uint8_t *rb = reinterpret_cast<uint8_t *>(s->ring);
  rb[k] = v;
  if (k < 64) rb[DF_RING + k] = v;
}
// dwords w and w + 1 of the ring (w < RING_ENT + 15: the mirror covers the wrap)
__device__ __forceinline__ uint2 ring_pair(const MatchShared *s, uint32_t w) {
  return make_uint2(s->ring[w], s->ring[w + 1]);
}
// dwords w .. w + N of the ring (w < RING_ENT, N <= 15: the mirror covers the wrap)
template <int N>
__device__ __forceinline__ void ring_dwords(const MatchShared *s, uint32_t w, uint32_t (&d)[N + 1]) {
#pragma unroll
  for (int k = 0; k <= N; ++k) d[k] = s->ring[w + k];
}
__device__ __forceinline__ uint32_t ld8(const MatchShared *s, uint32_t rel) {
  const uint32_t i = ridx(rel);
  return reinterpret_cast<const uint8_t *>(s->ring)[i];
}
// 4 bytes at any byte offset: an aligned dword pair and a byte align (an
// unaligned ds_read_b32 is legal on gfx950 but measured 25-45 % slower here)
__device__ __forceinline__ uint32_t ld32(const MatchShared *s, uint32_t rel) {
  const uint2 v = ring_pair(s, ridx(rel) >> 2);
  return __builtin_amdgcn_alignbyte(v.y, v.x, rel);  // (v_alignbyte_b32 reads the shift's low 2 bits only)
}
// chain key at p: the first klen bytes (kmask: bytes 0-3, kmask2: bytes 4-7)
struct Key {
  uint32_t kmask, kmask2;
};
__device__ __forceinline__ uint32_t key_hash(const MatchShared *s, uint32_t p, Key k) {
  // branch-free (a uniform branch here makes the compiler wait for each load)
  const uint32_t v = (ld32(s, p) & k.kmask) ^ ((ld32(s, p + 4) & k.kmask2) * 0x2545F491u);
  return __umulhi(v * 0x9E3779B1u, DF_HSIZE);
}
__device__ __forceinline__ uint32_t key4_hash(const MatchShared *s, uint32_t p) {
  return __umulhi(ld32(s, p) * 0x9E3779B1u, DF_H4SIZE);
}

// bytes [rel0, rel0 + len) of the super-chunk into the ring (len <= DF_SUB, rel0 % DF_SUB == 0)
__device__ void load_sub(MatchShared *s, const uint8_t *g, uint32_t rel0, uint32_t len) {
  const uint32_t t = threadIdx.x;
  const uint32_t k0 = ridx(rel0);  // multiple of DF_SUB
  if (len == DF_SUB && (reinterpret_cast<uintptr_t>(g) & 3) == 0) {
    ring_put32(s, (k0 >> 2) + t, reinterpret_cast<const uint32_t *>(g)[t]);
    return;
  }
  for (uint32_t i = t; i < len; i += DF_THREADS) ring_put8(s, k0 + i, g[i]);
}

// chain links for positions [lo, hi) (rel coords), by one wave, in position
// order: per step of 64 positions one LDS exchange head[h] <-> p.  The LDS
// applies the conflicting lanes of one exchange in lane order (checked on
// gfx950 by tools/micro/lds_xchg_order.hip), so each lane gets the newest
// earlier position of its bucket -- in its step or before -- and the head
// ends at the step's last one.  Exchanges of later steps are issued without
// waiting for earlier results (the wave's LDS operations stay in order); the
// progress is published for the searching waves (match_kernel).  T = 0: the
// 8-byte-key chains (head -> prev, s->linked); T = 1, by a second wave at the
// same time: the 4-byte-key table (head4 -> link4, s->linked4).
// Hashes of the keys at positions [lo, hi), by all threads of the workgroup,
// parked in the slots their links will fill: prev[ridx(p)] (the ring slot of
// p held a position 32 KiB back, out of every walk's reach) and
// link4[p % DF_SUB] (the previous sub-chunk's, whose searches are done).  The
// serial link waves then only read them (chain_link).
// Four consecutive positions per thread: three aligned dword reads (lanes on
// consecutive words: no bank conflicts) give all four 8-byte keys by byte
// aligns, and a full quad's hashes go out as one 8-byte store per table
// (one position per thread took two unaligned reads -- two dwords each -- and
// two 2-byte stores per position).  Slots outside [lo, hi) keep their values:
// below lo are links already made, and link4's slots past hi are this
// sub-chunk's first positions.
__device__ __forceinline__ void hash_keys(MatchShared *s, uint32_t lo, uint32_t hi, Key key) {
#ifdef ZT_DF_HASH1
  for (uint32_t p = lo + threadIdx.x; p < hi; p += DF_THREADS) {
    s->prev[ridx(p)] = (uint16_t)key_hash(s, p, key);
    s->link4[p & (DF_SUB - 1)] = (uint16_t)key4_hash(s, p);
  }
#else
  for (uint32_t p4 = (lo & ~3u) + 4 * threadIdx.x; p4 < hi; p4 += 4 * DF_THREADS) {
    const uint32_t w = ridx(p4) >> 2;  // (the mirror past the ring's end holds w + 1, w + 2 at the wrap)
    const uint2 d01 = ring_pair(s, w), d12 = ring_pair(s, w + 1);
    const uint32_t d0 = d01.x, d1 = d01.y, d2 = d12.y;
    uint32_t hk[4], h4[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint32_t x0 = k ? __builtin_amdgcn_alignbyte(d1, d0, k) : d0;
      const uint32_t x1 = k ? __builtin_amdgcn_alignbyte(d2, d1, k) : d1;
      const uint32_t v = (x0 & key.kmask) ^ ((x1 & key.kmask2) * 0x2545F491u);
      hk[k] = __umulhi(v * 0x9E3779B1u, DF_HSIZE);
      h4[k] = __umulhi(x0 * 0x9E3779B1u, DF_H4SIZE);
    }
    if (p4 >= lo && p4 + 4 <= hi) {
      *reinterpret_cast<uint2 *>(&s->prev[ridx(p4)]) = make_uint2(hk[0] | hk[1] << 16, hk[2] | hk[3] << 16);
      *reinterpret_cast<uint2 *>(&s->link4[p4 & (DF_SUB - 1)]) = make_uint2(h4[0] | h4[1] << 16, h4[2] | h4[3] << 16);
    } else {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        if (p4 + k >= lo && p4 + k < hi) {
          s->prev[ridx(p4 + k)] = (uint16_t)hk[k];
          s->link4[(p4 + k) & (DF_SUB - 1)] = (uint16_t)h4[k];
        }
      }
    }
  }
#endif
}

#ifndef ZT_CL_U
#define ZT_CL_U 8
#endif
constexpr int CL_U = ZT_CL_U;  // steps per group: hashes, then exchanges, then links
template <int T>
__device__ void chain_link(MatchShared *s, uint32_t lo, uint32_t hi, Key key) {
  const int lane = threadIdx.x & 63;
  const uint32_t nsteps = (hi - lo + 63) / 64;
  uint32_t hq[CL_U];
  // the keys' hashes were computed by every thread beforehand (hash_keys)
  // and parked in the slots the links are about to fill
  auto hashes = [&](uint32_t sb, uint32_t (&h)[CL_U]) {
#pragma unroll
    for (int j = 0; j < CL_U; ++j) {
      const uint32_t p = lo + (sb + j) * 64 + lane;
      const uint32_t pc = p < hi ? p : lo;  // (lanes past hi: any bucket, they exchange with a dummy)
      h[j] = T == 0 ? (uint32_t)s->prev[ridx(pc)] : (uint32_t)s->link4[pc & (DF_SUB - 1)];
    }
  };
  hashes(0, hq);
  for (uint32_t sb = 0; sb < nsteps; sb += CL_U) {
    // branch-free: lanes past hi exchange with / link into a dummy word, so
    // the compiler keeps every load and exchange of the group in flight
    uint32_t old[CL_U];
#ifdef ZT_DF_HEAD16
    if (T == 0) {
      // u16 heads: a masked-OR exchange of one half-word (ds_mskor_rtn_b32
      // applies a wave's conflicting lanes in lane order, as the exchange
      // does: tools/micro/lds_mskor_order.hip); the waits come after all CL_U
      // are issued (the compiler does not see inline-asm LDS operations)
      uint32_t sh[CL_U];
#pragma unroll
      for (int j = 0; j < CL_U; ++j) {
        const uint32_t p = lo + (sb + j) * 64 + lane;
        uint32_t *hp = p < hi ? &s->head[hq[j] >> 1] : &s->dummy[T];
        sh[j] = (hq[j] & 1) * 16;
        const uint32_t a = (uint32_t)(uintptr_t)hp, clr = 0xFFFFu << sh[j], set = (p & 0xFFFFu) << sh[j];
        __asm__ volatile("ds_mskor_rtn_b32 %0, %1, %2, %3" : "=v"(old[j]) : "v"(a), "v"(clr), "v"(set) : "memory");
      }
      static_assert(CL_U == 8, "the wait below names 8 results");
      __asm__ volatile("s_waitcnt lgkmcnt(0)"
                       : "+v"(old[0]), "+v"(old[1]), "+v"(old[2]), "+v"(old[3]), "+v"(old[4]), "+v"(old[5]),
                         "+v"(old[6]), "+v"(old[7])::"memory");
#pragma unroll
      for (int j = 0; j < CL_U; ++j) {
        const uint32_t p = lo + (sb + j) * 64 + lane;
        // (the distance modulo 2^16 is exact: stale heads are re-aged by head_sweep)
        old[j] = p - ((p - (old[j] >> sh[j])) & 0xFFFFu);
      }
    } else
#endif
    {
#pragma unroll
      for (int j = 0; j < CL_U; ++j) {
        const uint32_t p = lo + (sb + j) * 64 + lane;
        uint32_t *hp = p < hi ? (T == 0 ? &s->head[hq[j]] : &s->head4[hq[j]]) : &s->dummy[T];
        old[j] = atomicExch(hp, p);
      }
    }
    hashes(sb + CL_U, hq);
#pragma unroll
    for (int j = 0; j < CL_U; ++j) {
      const uint32_t p = lo + (sb + j) * 64 + lane;
      const uint32_t d = p - old[j];
      uint16_t *pp = p < hi ? (T == 0 ? &s->prev[ridx(p)] : &s->link4[p & (DF_SUB - 1)])
                            : reinterpret_cast<uint16_t *>(&s->dummy[2 + T]);
      *pp = (uint16_t)(d <= (uint32_t)DF_MAXDIST ? d : 0u);
    }
    const uint32_t done = lo + (sb + CL_U) * 64;
    if (lane == 0)
      __hip_atomic_store(T == 0 ? &s->linked : &s->linked4, done < hi ? done : hi, __ATOMIC_RELEASE,
                         __HIP_MEMORY_SCOPE_WORKGROUP);
  }
}

#ifdef ZT_DF_HEAD16
// u16 heads hold rel positions modulo 2^16: every HEAD_SWEEP sub-chunks, at
// rel position S (before that sub-chunk is linked), a head that is out of
// reach (age > DF_MAXDIST, and not one of the <= DF_HEAD positions linked
// ahead of S) is re-aged to S - 32768: until the next sweep it reads as
// 32768..61440 back -- never a link -- and a head in reach stays below 2^16
// back until then, so every link the exchange computes is the true distance.
constexpr uint32_t HEAD_SWEEP = 4;
static_assert(DF_MAXDIST + (HEAD_SWEEP + 1) * DF_SUB + DF_HEAD < 65536 - 1024, "ages stay below 2^16");
__device__ __forceinline__ void head_sweep(MatchShared *s, uint32_t S) {
  const uint32_t stale = (S - 32768u) & 0xFFFFu;
  for (uint32_t i = threadIdx.x; i < DF_HSIZE / 2; i += DF_THREADS) {
    const uint32_t w = s->head[i];
    uint32_t r = w;
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const uint32_t age = (S - (w >> (16 * k))) & 0xFFFFu;
      if (age > (uint32_t)DF_MAXDIST && age < 65536u - 1024u) r = (r & ~(0xFFFFu << (16 * k))) | (stale << (16 * k));
    }
    if (r != w) s->head[i] = r;
  }
}
#endif

// 4 bytes at byte x of a register window (x a compile-time constant after unrolling)
template <int X>
__device__ __forceinline__ uint32_t win32(const uint32_t (&w)[9]) {
  return (X & 3) ? __builtin_amdgcn_alignbyte(w[(X >> 2) + 1], w[X >> 2], X & 3) : w[X >> 2];
}

constexpr int DF_NEAR = 16;  // near distances probed from registers

// matches shorter than the chain key at distances 1..probe, from a register
// window of bytes [pb - 16, pb + 16): longest wins, ties to the nearest
template <int K, int D>
__device__ __forceinline__ void near_probe(const uint32_t (&w)[9], uint32_t cur0, uint32_t cur1, uint32_t p,
                                           uint32_t max_len, int probe, uint32_t &best_len, uint32_t &best_dist) {
  if constexpr (D <= DF_NEAR) {
    if (D <= probe && (uint32_t)D <= p) {
      const uint32_t m0 = win32<16 + K - D>(w) ^ cur0;
      if ((m0 & 0xFFFFFFu) == 0) {
        uint32_t len;
        if (m0) {
          len = 3;
        } else {
          const uint32_t m1 = win32<20 + K - D>(w) ^ cur1;
          len = m1 ? 4 + ((uint32_t)(__ffs(m1) - 1) >> 3) : 8;
        }
        if (len > max_len) len = max_len;
        if (len > best_len) {
          best_len = len;
          best_dist = D;
        }
      }
    }
    near_probe<K, D + 1>(w, cur0, cur1, p, max_len, probe, best_len, best_dist);
  }
}

// Branch-free prefilter of the near probes of position pb + K: the minimum
// over distances 1..DF_NEAR of (3 bytes at p - D) XOR (3 bytes at p) is zero
// iff some distance has a 3-byte match (out-of-range distances only give
// false positives; near_probe re-checks).  One alignbyte + bitop3 + min per
// distance instead of a compare-and-branch per distance.
template <int K, int D>
__device__ __forceinline__ uint32_t near_any(const uint32_t (&w)[9], uint32_t cur0, uint32_t m) {
  if constexpr (D <= DF_NEAR) {
    const uint32_t x = (win32<16 + K - D>(w) ^ cur0) & 0xFFFFFFu;
    return near_any<K, D + 1>(w, cur0, m < x ? m : x);
  } else {
    return m;
  }
}

// One position's hash-chain walk (newest candidate first).  Two walks are
// interleaved per thread so that their dependent LDS loads overlap.
struct Walk {
  uint32_t p, q, link, max_len, best_len, best_dist, o, pw, omask, cur, cur2, cur3, cur4;
  uint32_t cl;  // carried match length (kept unless the walk finds one at least as long, nearer)
  int max_hops;  // (hops taken = the pair loop's step count while the walk is active)
  uint32_t late; // improvements found at hop >= P.adapt_depth (low half) / adapt_depth2 (high half)
  bool active;
};

// n words at byte rel of the ring, unaligned (the 64-byte mirror past the
// ring's end keeps up to 15 words contiguous): n + 1 dword loads, no wrap math
template <int N>
__device__ __forceinline__ void ld_run(const MatchShared *s, uint32_t rel, uint32_t (&o)[N]) {
  const uint32_t w = ridx(rel) >> 2, sh = rel;  // (v_alignbyte_b32 reads the shift's low 2 bits only)
  uint32_t d[N + 1];
  ring_dwords<N>(s, w, d);
#pragma unroll
  for (int k = 0; k < N; ++k) o[k] = __builtin_amdgcn_alignbyte(d[k + 1], d[k], sh);
}

// start the walk of position p (carry: the previous position's match); cur..cur4
// are bytes 0..15 of p
__device__ __forceinline__ void walk_init(Walk &w, const MatchShared *s, const DeflateParams &P, uint32_t p, uint32_t p1,
                                          uint32_t cur, uint32_t cur2, uint32_t cur3, uint32_t cur4,
                                          uint32_t carry_len, uint32_t carry_dist, uint32_t link, int mc) {
  w.p = p;
  w.q = p;
  w.cur = cur;
  w.cur2 = cur2;
  w.cur3 = cur3;
  w.cur4 = cur4;
  w.max_len = p < p1 ? ((p1 - p) < 258 ? (p1 - p) : 258) : 0;
  w.best_len = 0;
  w.best_dist = 0;
  if (carry_len > 3 && w.max_len >= 3) {
    w.best_len = carry_len - 1 < w.max_len ? carry_len - 1 : w.max_len;
    w.best_dist = carry_dist;
  }
  w.max_hops = (int)w.best_len >= P.good ? (mc >> 2) : mc;
  w.active = w.max_len >= (uint32_t)P.klen && (int)w.best_len < P.skip_len;
  w.cl = w.best_len;
#ifdef ZT_DF_CARRY_TIES
  // the walk visits the nearest candidates first: one as long as the carried
  // match is found before the carried distance and costs fewer distance bits
  if (w.best_len >= 4) w.best_len -= 1;
#endif
  // one word per hop filters the candidates: the word ending at best_len (a
  // candidate can only win if it matches there), or before any match the
  // first bytes of the key (the chains' hash buckets also hold collisions)
  w.o = w.best_len >= 4 ? w.best_len - 3 : 0;
  w.omask = w.best_len >= 4 || P.klen >= 4 ? 0xFFFFFFFFu : 0xFFFFFFu;
  w.pw = cur;
  w.link = 0;
  if (w.active) {
    if (w.best_len >= 4) w.pw = ld32(s, p + w.o);
    w.link = link;  // prev[ridx(p)], read by search_quad with its three neighbours
    w.active = w.link != 0;
  }
}

// equal leading bytes (0..16) of four XORed words: the first differing bit
// of each word (v_ffbl: ~0 for none), offset by the word's place with
// unsigned saturation (none stays ~0; the last word's by a min with 32, so
// that no constant needs a register), the least of them -- 11 VALU (round
// 4's per-word selects: 17, and the measurement is the walk's VALU-heaviest
// part: match 22.4 -> 20.4 ms per GiB, streams identical); inline asm because
// the compiler rewrites ffs of a possibly-zero word into compares and selects
__device__ __forceinline__ uint32_t ffbl_raw(uint32_t x) {
  uint32_t r;
  asm("v_ffbl_b32 %0, %1" : "=v"(r) : "v"(x));
  return r;
}
template <uint32_t B>
__device__ __forceinline__ uint32_t add_sat(uint32_t a) {
  uint32_t r;
  static_assert(B <= 64, "an inline constant (VOP3 takes no literal here)");
  asm("v_add_u32_e64 %0, %1, %2 clamp" : "=v"(r) : "v"(a), "i"(B));
  return r;
}
__device__ __forceinline__ uint32_t min3_u32(uint32_t a, uint32_t b, uint32_t c) {
  uint32_t r;
  asm("v_min3_u32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}
__device__ __forceinline__ uint32_t eq_len16(uint32_t x0, uint32_t x1, uint32_t x2, uint32_t x3) {
  const uint32_t m = min3_u32(ffbl_raw(x0), add_sat<32>(ffbl_raw(x1)), add_sat<64>(ffbl_raw(x2)));
  const uint32_t l3 = min(ffbl_raw(x3), 32u) + 96u;  // (<= 128: all 16 bytes equal)
  return min(m, l3) >> 3;
}

// a candidate q that passed the one-word filter: its length from byte 0
// (the filter checked at most 4 bytes) and keep the longest
__device__ __forceinline__ void walk_extend(Walk &w, const MatchShared *s, const DeflateParams &P, uint32_t q,
                                            uint32_t late) {
#ifdef ZT_DF_COUNT
  atomicAdd(&g_df_count[2], 1ull);
  // (wave-level executions of the measurement: its first active lane counts)
  if ((int)(threadIdx.x & 63) == __ffsll((unsigned long long)__ballot(1)) - 1) atomicAdd(&g_df_count[3], 1ull);
#endif
  // the first 16 bytes: q's words in one run of loads, p's from registers;
  // lengths branch-free, so that every load of the run is in flight at once
  uint32_t qw[4];
  ld_run<4>(s, q, qw);
  uint32_t len = eq_len16(qw[0] ^ w.cur, qw[1] ^ w.cur2, qw[2] ^ w.cur3, qw[3] ^ w.cur4);
  // all 16 matched: 16 more bytes per round until a mismatch (or max_len)
  bool more = len == 16;
  while (more && len < w.max_len) {
    uint32_t qx[4], px[4];
    ld_run<4>(s, q + len, qx);
    ld_run<4>(s, w.p + len, px);
    const uint32_t l = eq_len16(qx[0] ^ px[0], qx[1] ^ px[1], qx[2] ^ px[2], qx[3] ^ px[3]);
    len += l;
    more = l == 16;
  }
  if (len > w.max_len) len = w.max_len;
  // branch-free update (selects instead of nested exec-mask branches: the
  // pass runs with a few lanes of the wave, and every branch of the nest is
  // taken by one of them: match 21.0 -> 20.3 ms per GiB, streams identical)
  const bool upd = len >= 3 && len > w.best_len;
#ifdef ZT_DF_COUNT
  atomicAdd(&g_df_count[upd ? 4 : 6], 1ull);
  if (len < 8) atomicAdd(&g_df_count[5], 1ull);
#endif
  const bool stop = upd && ((int)len >= P.nice_len || len >= w.max_len);
  const bool newo = upd && !stop && len >= 4;
  w.late += upd ? late : 0u;
  w.best_len = upd ? len : w.best_len;
  w.best_dist = upd ? w.p - q : w.best_dist;
  w.active = w.active && !stop;
  w.o = newo ? len - 3 : w.o;
  w.omask = newo ? 0xFFFFFFFFu : w.omask;
  const uint32_t npw = ld32(s, w.p + w.o);
  w.pw = newo ? npw : w.pw;
}



// one hop of two walks: every LDS load of both hops is issued before any is
// used (the walks are latency-bound pointer chases), then the checks.  Per
// hop two loads: the link and the filter word.
// `step`: the pair loop's count of steps before this one (wave-uniform): an
// active walk has taken exactly that many hops.  Inactive walks keep
// stepping through stale links: their loads stay inside the ring and are
// never used.
__device__ __forceinline__ void walk_pair_step(Walk &a, Walk &b, const MatchShared *s, const DeflateParams &P,
                                               int step) {
  const uint32_t qa = a.q - a.link;
  const uint32_t qb = b.q - b.link;
  const bool ha = a.active && a.p - qa <= (uint32_t)DF_MAXDIST;
  const bool hb = b.active && b.p - qb <= (uint32_t)DF_MAXDIST;
  const uint32_t la = s->prev[ridx(qa)], lb = s->prev[ridx(qb)];
  const uint32_t oa = ld32(s, qa + a.o), ob = ld32(s, qb + b.o);
  a.q = qa;
  b.q = qb;
#ifdef ZT_DF_COUNT
  if ((threadIdx.x & 63) == 0) atomicAdd(&g_df_count[0], 1ull);
  atomicAdd(&g_df_count[1], (unsigned long long)(ha ? 1 : 0) + (hb ? 1 : 0));
#endif
  // (& not &&: a short-circuit lets the compiler sink a filter read into a
  // branch, behind the other walk's wait)
  const bool ca = ha & (((oa ^ a.pw) & a.omask) == 0);
  const bool cb = hb & (((ob ^ b.pw) & b.omask) == 0);
  a.link = la;
  b.link = lb;
  a.active = ha && la != 0 && step + 1 < a.max_hops;
  b.active = hb && lb != 0 && step + 1 < b.max_hops;
#if defined(ZT_DF_X_EXT0)
  // (measurement build: candidates measured at the first hop only -- wrong
  // streams; the time without the later, divergent measurement passes)
  if (ca && step == 0) walk_extend(a, s, P, qa, 0);
  if (cb && step == 0) walk_extend(b, s, P, qb, 0);
#else
  const uint32_t late = (P.adapt_depth && step >= P.adapt_depth ? 1u : 0u) |
                        (P.adapt_depth2 && step >= P.adapt_depth2 ? 0x10000u : 0u);
  if (ca) walk_extend(a, s, P, qa, late);
  if (cb) walk_extend(b, s, P, qb, late);
#endif
}


// finish position pb + K when the chain found nothing of the key's length:
// the near probes, then the newest earlier position with the same 4 bytes
// (the 4-byte-key table; the chains' 8-byte keys miss the 4..7-byte matches
// that make up much of source text)
template <int K>
__device__ __forceinline__ uint32_t walk_finish(const Walk &w, const MatchShared *s, const DeflateParams &P,
                                                const uint32_t (&win)[9], uint32_t near, uint32_t lim4, uint32_t d4,
                                                uint32_t &carry_len, uint32_t &carry_dist) {
  uint32_t best_len = w.best_len < w.cl ? w.cl : w.best_len, best_dist = w.best_dist;
  // a far 3-byte match (carried from the previous position) is dropped in
  // the end: it must not hide a near one
  if (best_len == 3 && best_dist > (uint32_t)P.too_far) best_len = 0;
  const bool short_ = best_len < (uint32_t)P.klen;
  if (near == 0 && w.max_len >= 3 && short_)
    near_probe<K, 1>(win, w.cur, w.cur2, w.p, w.max_len, P.probe, best_len, best_dist);
#ifndef ZT_DF_NOP4
  // (positions from lim4 on have no 4-byte link: their keys would need bytes
  // past the segment's end)
  if (w.max_len >= 4 && short_ && w.p < lim4) {
    uint32_t qw[2];
    ld_run<2>(s, w.p - d4, qw);
    const uint32_t x0 = qw[0] ^ w.cur, x1 = qw[1] ^ w.cur2;
    uint32_t len = x0 ? 0u : 4 + min((uint32_t)(__ffs(x1) - 1) >> 3, 4u);
    len = len < w.max_len ? len : w.max_len;
    // a far match must be longer by two bytes than a near one to replace it
    // (its distance code costs more than the byte it gains)
    const uint32_t need = best_len + (best_len >= 3 && d4 > (uint32_t)P.too_far ? 2u : 1u);
    if (d4 != 0 && len >= 4 && len >= need && (len > 4 || d4 <= (uint32_t)ZT_DF_P4FAR)) {
      best_len = len;
      best_dist = d4;
    }
  }
#endif
  carry_len = best_len;
  carry_dist = best_dist;
  if (best_len == 3 && best_dist > (uint32_t)P.too_far) best_len = 0;
  return best_len >= 3 ? res_pack(0, best_len, best_dist) : 0u;
}

// longest match for positions [pb, pb + 4) of the sub-chunk [p0, p1) -> res_out[p - p0];
// matches end at pml (>= p1)
__device__ void search_quad(const MatchShared *s, const DeflateParams &P, uint32_t pb, uint32_t p0, uint32_t p1,
                            uint32_t pml, uint32_t lim4, Key key, uint32_t *res_out, int mc, uint32_t &late) {
  if (pb >= p1) return;
  // bytes [pb - 16, pb + 20) (pb is a multiple of 4; before rel 0 the words
  // are never used: near distances stay <= p)
  uint32_t w[9];
  ring_dwords<8>(s, ridx(pb - 16) >> 2, w);
  // the four positions' 4-byte-table links (final: the super-step waited for
  // them), read with the window so that walk_finish's lookups start from
  // the candidate's bytes -- one LDS round trip each instead of two
  const uint2 l4 = *reinterpret_cast<const uint2 *>(&s->link4[pb & (DF_SUB - 1)]);
  // (and the four chain links the walks start from: positions 1 and 3 begin
  // after 0 and 2 finish, their first link already in registers)
  const uint2 l8 = *reinterpret_cast<const uint2 *>(&s->prev[ridx(pb)]);
  // positions 0 and 2 walk together, then 1 and 3 with the carry of 0 and 2
  uint32_t out[4];
  uint32_t c0l, c0d, c2l, c2d, cl, cd;
  const uint32_t nr0 = near_any<0, 1>(w, win32<16>(w), ~0u), nr1 = near_any<1, 1>(w, win32<17>(w), ~0u);
  const uint32_t nr2 = near_any<2, 1>(w, win32<18>(w), ~0u), nr3 = near_any<3, 1>(w, win32<19>(w), ~0u);
  Walk wa, wb;
  wa.late = wb.late = 0;
  walk_init(wa, s, P, pb, pml, win32<16>(w), win32<20>(w), win32<24>(w), win32<28>(w), 0, 0, l8.x & 0xFFFFu, mc);
  walk_init(wb, s, P, pb + 2, pml, win32<18>(w), win32<22>(w), win32<26>(w), win32<30>(w), 0, 0, l8.y & 0xFFFFu, mc);
  for (int step = 0; wa.active || wb.active; ++step) walk_pair_step(wa, wb, s, P, step);
  out[0] = walk_finish<0>(wa, s, P, w, nr0, lim4, l4.x & 0xFFFFu, c0l, c0d);
  out[2] = walk_finish<2>(wb, s, P, w, nr2, lim4, l4.y & 0xFFFFu, c2l, c2d);
#ifdef ZT_DF_NOCARRY  // experiment: positions 1 and 3 start without the carried match
  c0l = c0d = c2l = c2d = 0;
#endif
  walk_init(wa, s, P, pb + 1, pml, win32<17>(w), win32<21>(w), win32<25>(w), win32<29>(w), c0l, c0d, l8.x >> 16, mc);
  walk_init(wb, s, P, pb + 3, pml, win32<19>(w), win32<23>(w), win32<27>(w), win32<31>(w), c2l, c2d, l8.y >> 16, mc);
  for (int step = 0; wa.active || wb.active; ++step) walk_pair_step(wa, wb, s, P, step);
  late += wa.late + wb.late;
  out[1] = walk_finish<1>(wa, s, P, w, nr1, lim4, l4.x >> 16, cl, cd);
  out[3] = walk_finish<3>(wb, s, P, w, nr3, lim4, l4.y >> 16, cl, cd);
  // the positions' own bytes (res_pack)
  out[0] |= win32<16>(w) << 24;
  out[1] |= win32<17>(w) << 24;
  out[2] |= win32<18>(w) << 24;
  out[3] |= win32<19>(w) << 24;
  if (pb + 4 <= p1) {
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    u32x4 v = {out[0], out[1], out[2], out[3]};
    *reinterpret_cast<u32x4 *>(res_out + (pb - p0)) = v;
  } else {
    for (uint32_t k = 0; k < 4 && pb + k < p1; ++k) res_out[pb - p0 + k] = out[k];
  }
}

__global__ __launch_bounds__(DF_THREADS) void match_kernel(DeflateParams P) {
  __shared__ MatchShared s;
  const uint32_t t = threadIdx.x;
  // workgroups go to the 8 XCDs round robin, and every 8th super-chunk starts
  // a segment (no history: 18 % fewer positions): rotate each group of 8 so
  // that every XCD gets its share of those
  uint32_t wg = blockIdx.x;
  if ((wg | 7u) < gridDim.x) wg = (wg & ~7u) | ((wg + (wg >> 3)) & 7u);
  const bool big = wg < P.big_wgs;
  const uint32_t b0 = big ? wg * P.blocks_per_wg : P.big_wgs * P.blocks_per_wg + (wg - P.big_wgs) * P.tail_k;
  const uint32_t kb = big ? P.blocks_per_wg : P.tail_k;
  const uint32_t b1 = (b0 + kb) < P.nblocks ? (b0 + kb) : P.nblocks;
  if (P.store) {  // every block of the super-chunk goes stored: nothing to search
    bool all = true;
    for (uint32_t b = b0; b < b1; ++b) all = all && P.store[b];
    if (all) return;
  }
  // (batch: a workgroup's blocks belong to one stream, which starts at f_lo)
  const uint64_t f_lo = P.span ? P.halo + P.span[2 * (uint64_t)b0] : 0;
  const uint64_t f_end = P.span ? P.halo + P.span[2 * (uint64_t)b0 + 1] : P.end;
  const uint64_t s_lo = P.halo + (uint64_t)b0 * DF_BLOCK;
  const uint64_t s_hi = (P.halo + (uint64_t)b1 * DF_BLOCK) < f_end ? (P.halo + (uint64_t)b1 * DF_BLOCK) : f_end;
  // a segment start (restart point) sees no history: its matches stay inside
  // the segment, so inflate can decode segments independently
  const bool restart = P.span ? (((s_lo - f_lo) / DF_BLOCK) % P.restart) == 0
                              : (b0 % P.restart) == 0 && (b0 > 0 || P.halo == 0);
  // history: whole sub-chunks, so that the searched range starts on a sub-chunk
  const uint64_t hmax = P.hist_max;
  const uint64_t hist = restart ? 0 : ((s_lo - f_lo) < hmax ? ((s_lo - f_lo) & ~uint64_t(DF_SUB - 1)) : hmax);
  const uint64_t h_lo = s_lo - hist;
  const uint8_t *g = P.base + h_lo;  // rel 0
  const uint32_t rs = (uint32_t)(s_lo - h_lo), re = (uint32_t)(s_hi - h_lo);
  // bytes available for hashing: the stream's, but not past the end of the
  // super-chunk's segment (a restart point): positions near a segment end
  // are never linked, so a segment is searched alike whether the stream goes
  // on or ends there (a shard, a pipeline piece, zt_shard.py)
  const bool seg_end = s_hi == f_end || (P.span ? ((s_hi - f_lo) / DF_BLOCK) % P.restart == 0
                                                 : ((s_hi - P.halo) / DF_BLOCK) % P.restart == 0);
  const uint32_t rend = seg_end ? (uint32_t)(s_hi - h_lo) : (uint32_t)(f_end - h_lo);
  Key key;
  key.kmask = P.klen >= 4 ? 0xFFFFFFFFu : 0xFFFFFFu;
  key.kmask2 = P.klen >= 8 ? 0xFFFFFFFFu : P.klen == 6 ? 0xFFFFu : P.klen == 5 ? 0xFFu : 0u;
  const uint32_t kext = (uint32_t)P.klen - 1;  // a key at p needs bytes up to p + kext

#ifdef ZT_DF_HEAD16
  for (uint32_t i = t; i < DF_HSIZE / 2; i += DF_THREADS) s.head[i] = 0x80008000u;  // (rel 0 - 32768: out of reach)
#else
  for (uint32_t i = t; i < DF_HSIZE; i += DF_THREADS) s.head[i] = kNoHead;
#endif
  for (uint32_t i = t; i < DF_H4SIZE; i += DF_THREADS) s.head4[i] = kNoHead;
  // the last kext positions of the first sub-chunk read link4 before any
  // link reached their slots: no candidate (not the LDS left by an earlier
  // workgroup, which made the output depend on the run)
  for (uint32_t i = t; i < DF_SUB; i += DF_THREADS) s.link4[i] = 0;
  __syncthreads();
  uint32_t inserted = 0;  // positions [0, inserted) are in the chains
  if (re > 0) load_sub(&s, g, 0, re < DF_SUB ? re : DF_SUB);
  // (the second sub-chunk's head: bytes [DF_SUB, DF_SUB + DF_HEAD); heads
  // run on past the super-chunk into the stream, so that a position at a
  // block end is linked and searched alike whatever the super-chunk size)
  if (DF_HEAD && t < (uint32_t)DF_HEAD && DF_SUB + t < rend) {
    ring_put8(&s, ridx(DF_SUB + t), g[DF_SUB + t]);
  }
  const bool g_aligned = (reinterpret_cast<uintptr_t>(g) & 3) == 0;
  for (uint32_t p0 = 0; p0 < re; p0 += DF_SUB) {
    const uint32_t p1 = (p0 + DF_SUB) < re ? (p0 + DF_SUB) : re;
    lds_barrier();
    [[maybe_unused]] uint64_t t0, t1, t2, t3;
    DF_T(t0);
    // bytes in the ring: the sub-chunk and the next one's head
    const uint32_t dend = DF_HEAD ? (p1 + DF_HEAD < rend ? p1 + DF_HEAD : rend) : p1;
    uint32_t ih = dend >= kext ? dend - kext : 0;
    if (ih > p1) ih = p1;
    if (rend >= kext && ih > rend - kext) ih = rend - kext;
    const bool link = ih > inserted;
    // per-block depth: the block's first sub-chunk (the probe) walks max_chain
    // hops and counts late improvements; its verdict holds for the rest of
    // the block (a function of the block's own positions: streams do not
    // depend on how blocks are grouped into workgroups)
    const bool probe_sub = p0 >= rs && ((p0 - rs) % DF_BLOCK) == 0;
    if (t == 0) {
      s.linked = link ? inserted : ih;
      s.linked4 = link ? inserted : ih;
      s.work = 0;
      if (p0 > rs && ((p0 - rs) % DF_BLOCK) == DF_SUB)  // (the probe's counts are complete: a barrier since)
        s.depth = P.adapt_depth && s.late * 4096u <= (uint32_t)P.adapt_thr * DF_SUB     ? P.adapt_depth
                  : P.adapt_depth2 && s.late2 * 4096u <= (uint32_t)P.adapt_thr2 * DF_SUB ? P.adapt_depth2
                                                                                          : P.max_chain;
      if (probe_sub) s.late = s.late2 = 0;
    }
    // the next sub-chunk is fetched while this one is searched
    const uint32_t n0 = p0 + DF_SUB;
    const bool fast = g_aligned && n0 + DF_SUB <= re;
    uint32_t nv = 0;
    if (fast) nv = reinterpret_cast<const uint32_t *>(g + n0)[t];
    // and the head of the one after it (written with nv, after the search)
    const uint32_t hd0 = n0 + DF_SUB;
    const bool hload = DF_HEAD && t < (uint32_t)DF_HEAD && hd0 + t < rend;
    uint8_t hb = 0;
    if (hload) hb = g[hd0 + t];
    // matches end at the block's end (or the data's)
    uint32_t pml = p1;
    if (DF_HEAD && p0 >= rs) {
      const uint32_t bend = rs + ((p0 - rs) / DF_BLOCK + 1) * DF_BLOCK;
      pml = bend < dend ? bend : dend;
    }
    if (link) hash_keys(&s, inserted, ih, key);
#ifdef ZT_DF_HEAD16
    if ((p0 / DF_SUB) % HEAD_SWEEP == 0 && link) head_sweep(&s, p0);
#endif
    lds_barrier();
    DF_T(t1);
    // wave 0 links the 8-byte-key chains and wave 1 the 4-byte-key table,
    // step by step; every wave (waves 0 and 1 once done) takes super-steps of
    // 256 positions in order and searches them as soon as their links are
    // final (positions only read links of older ones)
#ifdef ZT_DF_LINK_PRIO
    // the linking waves are on every searcher's critical path: issue first
    if (t < 128 && link) __builtin_amdgcn_s_setprio(ZT_DF_LINK_PRIO);
#endif
    if (t < 64 && link) chain_link<0>(&s, inserted, ih, key);
    if (t >= 64 && t < 128 && link) chain_link<1>(&s, inserted, ih, key);
#ifdef ZT_DF_LINK_PRIO
    if (t < 128 && link) __builtin_amdgcn_s_setprio(0);
#endif
#ifdef ZT_DF_TIME
    uint64_t tl;
    DF_T(tl);
    if ((t & 63) == 0 && t < 128 && link) atomicAdd(&g_df_time[4], (unsigned long long)(tl - t1));
    uint64_t t_wait = 0, t_srch = 0, n_ss = 0;
#endif
    inserted = link ? ih : inserted;
    if (p0 >= rs) {
      const uint32_t nss = (p1 - p0 + 255) / 256;
      const int mc = probe_sub || !P.adapt_depth ? P.max_chain : s.depth;
      uint32_t late = 0;
      uint32_t *res_out = P.res + (h_lo + p0 - P.halo);  // res[input pos]: rel r <-> input h_lo + r - halo
      for (;;) {
        uint32_t ss = 0;
        if ((t & 63) == 0) ss = atomicAdd(&s.work, 1u);
        ss = (uint32_t)__shfl((int)ss, 0, 64);
        if (ss >= nss) break;
        const uint32_t need = (p0 + 256 * (ss + 1)) < ih ? (p0 + 256 * (ss + 1)) : ih;
#ifdef ZT_DF_TIME
        uint64_t w0, w1, w2;
        DF_T(w0);
#endif
        while (min(__hip_atomic_load(&s.linked, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP),
                   __hip_atomic_load(&s.linked4, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP)) < need)
          __builtin_amdgcn_s_sleep(1);
#ifdef ZT_DF_TIME
        DF_T(w1);
#endif
        search_quad(&s, P, p0 + 256 * ss + 4 * (t & 63), p0, p1, pml, ih, key, res_out, mc, late);
#ifdef ZT_DF_TIME
        DF_T(w2);
        t_wait += w1 - w0;
        t_srch += w2 - w1;
        n_ss += 1;
#endif
      }
      if (probe_sub && P.adapt_depth) {
        // (per wave each half stays below 2^16: 256 positions x < 20 hops)
        for (int o = 32; o; o >>= 1) late += (uint32_t)__shfl_xor((int)late, o, 64);
        if ((t & 63) == 0 && (late & 0xFFFFu)) atomicAdd(&s.late, late & 0xFFFFu);
        if ((t & 63) == 0 && (late >> 16)) atomicAdd(&s.late2, late >> 16);
      }
    }
    DF_T(t2);
    lds_barrier();
    DF_T(t3);
#ifdef ZT_DF_TIME
    // per wave (lane 0): hash phase, searching, barrier wait, (wave, sub-chunk)
    // pairs, link waits, super-steps, link + search loop
    if ((t & 63) == 0) {
      atomicAdd(&g_df_time[0], (unsigned long long)(t1 - t0));
      atomicAdd(&g_df_time[1], (unsigned long long)t_srch);
      atomicAdd(&g_df_time[2], (unsigned long long)(t3 - t2));
      atomicAdd(&g_df_time[3], 1ull);
      atomicAdd(&g_df_time[5], (unsigned long long)t_wait);
      atomicAdd(&g_df_time[6], (unsigned long long)n_ss);
      atomicAdd(&g_df_time[7], (unsigned long long)(t2 - t1));
    }
#endif
    if (fast) {
      ring_put32(&s, (ridx(n0) >> 2) + t, nv);
    } else if (n0 < re) {
      load_sub(&s, g + n0, n0, (re - n0) < DF_SUB ? (re - n0) : DF_SUB);
    }
    if (hload) {
      ring_put8(&s, ridx(hd0 + t), hb);
    }
  }
}

// ================================ 2. block_kernel ================================
constexpr int PM_MAX = 2 * 286;  // package-merge list length bound (2m - 2)
struct HufScratch {
  uint32_t key[320];              // (freq << 9) | symbol, sorted ascending (the first m are used)
  uint32_t lst[2][PM_MAX];        // package-merge lists (weights), ping-pong
  uint32_t pkg[14][PM_MAX / 32];  // per level: which list entries are packages
  uint32_t items[16];             // selected items per level
  uint32_t bl_count[16];
};

// parse staging ring (parse_block_dma)
constexpr int PB_CH = 4;
#ifndef ZT_PB_NCH
#define ZT_PB_NCH 4
#endif
constexpr int PB_NCH = ZT_PB_NCH;
constexpr int PB_LOADS = PB_CH;  // global_load_lds per chunk (res words; the bytes ride in res)
struct ParseStage {
  uint32_t res[PB_NCH][PB_CH * 64];
};

struct BlockShared {
  uint32_t lit_hist[288];
  uint32_t dist_hist[32];
  uint32_t n_cl_syms, hlit, hdist, hclen;
  union {
    struct {
      uint32_t lit_code[288];
      uint32_t dist_code[32];
      uint32_t cl_code[19];
      uint8_t lit_len[288];
      uint8_t dist_len[32];
      uint8_t cl_len[20];
      uint16_t cl_syms[320];  // sym | extra_value << 5
      HufScratch huf;
    };
  };
};

// One wave per workgroup: LDS operations of a wave complete in order, so a
// hand-off between lanes only needs the compiler not to reorder.
__device__ __forceinline__ void wsync() {
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
}

// freq[0..n) -> len[0..n), limited to `limit` bits.  Always produces a complete
// code with >= 2 symbols (zlib's rule), forcing symbols 0/1 in when needed.
// ascending bitonic sort of 64 * R keys held R per lane (key index lane * R + r):
// partners inside a lane are register swaps, others one cross-lane shuffle
template <int R>
__device__ __forceinline__ void reg_bitonic(uint32_t (&key)[R], int lane) {
  constexpr int N = 64 * R;
#pragma unroll
  for (int k = 2; k <= N; k <<= 1) {
#pragma unroll
    for (int j = k >> 1; j > 0; j >>= 1) {
      if (j < R) {
#pragma unroll
        for (int r = 0; r < R; ++r) {
          if ((r & j) == 0) {
            const uint32_t i = (uint32_t)lane * R + r;
            const bool up = (i & k) == 0;
            const uint32_t a = key[r], b = key[r | j];
            const bool sw = (a > b) == up;
            key[r] = sw ? b : a;
            key[r | j] = sw ? a : b;
          }
        }
      } else {
#pragma unroll
        for (int r = 0; r < R; ++r) {
          const uint32_t other = (uint32_t)__shfl_xor((int)key[r], j / R, 64);
          const uint32_t i = (uint32_t)lane * R + r;
          const bool up = (i & k) == 0;
          const bool lower = (i & j) == 0;
          const uint32_t mn = key[r] < other ? key[r] : other, mx = key[r] < other ? other : key[r];
          key[r] = (lower == up) ? mn : mx;
        }
      }
    }
  }
}

// keys (freq << 9 | symbol, or ~0 for unused) sorted ascending into h.key[0..)
template <int R>
__device__ __forceinline__ void sort_keys(HufScratch &h, const uint32_t *freq_in, int n, int lane) {
  uint32_t key[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int i = lane * R + r;
    const uint32_t f = i < n ? freq_in[i] : 0u;
    key[r] = (i < n && f) ? ((f << 9) | (uint32_t)i) : 0xFFFFFFFFu;
  }
  reg_bitonic<R>(key, lane);
#pragma unroll
  for (int r = 0; r < R; ++r)
    if (lane * R + r < 320) h.key[lane * R + r] = key[r];
}

__device__ void huff_lengths(BlockShared *s, const uint32_t *freq_in, int n, int limit, uint8_t *len_out) {
  const int lane = threadIdx.x & 63;
  HufScratch &h = s->huf;
  for (int i = lane; i < n; i += 64) len_out[i] = 0;
  wsync();
  uint32_t m = 0;
  for (int i = lane; i < n; i += 64) m += (freq_in[i] != 0);
  for (int off = 32; off; off >>= 1) m += __shfl_xor(m, off, 64);
  if (m < 2) {
    // a complete code needs two symbols (zlib rejects a lone one-bit code)
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
    wsync();
    return;
  }
  // sort by (frequency, symbol) in registers
  if (n <= 64)
    sort_keys<1>(h, freq_in, n, lane);
  else
    sort_keys<8>(h, freq_in, n, lane);
  wsync();
  // Length-limited optimal code lengths by package-merge, wave-parallel: the
  // level-j list is the items merged with the packages (pairs) of the level
  // j-1 list, kept to its first 2m - 2 entries; each merge by merge-path
  // (every lane a contiguous run of outputs after a binary search).  The
  // selection is then a prefix of every level: c_L = 2m - 2 entries at the
  // top, c_{j-1} = 2 x (packages among the first c_j), and item k's code
  // length is the number of levels whose selected prefix holds it.
  const uint32_t mm = m, cap = 2 * mm - 2;
  for (uint32_t i = lane; i < mm; i += 64) h.lst[0][i] = h.key[i] >> 9;
  for (int j = 0; j < limit - 1; ++j)
    for (uint32_t w = lane; w < PM_MAX / 32; w += 64) h.pkg[j][w] = 0;
  wsync();
  uint32_t lp = mm;  // length of the previous level's list
  for (int j = 1; j < limit; ++j) {
    const uint32_t *P = h.lst[(j - 1) & 1];
    uint32_t *Q = h.lst[j & 1];
    const uint32_t np = lp / 2;
    const uint32_t lq = mm + np < cap ? mm + np : cap;
    auto A = [&](uint32_t i) -> uint32_t { return h.key[i] >> 9; };
    auto B = [&](uint32_t i) -> uint32_t { return P[2 * i] + P[2 * i + 1]; };
    const uint32_t per = (lq + 63) / 64;
    const uint32_t d = (uint32_t)lane * per;
    if (d < lq) {
      // merge path: a = items among the first d outputs (items first on ties)
      uint32_t lo = d > np ? d - np : 0, hi = d < mm ? d : mm;
      while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (A(mid) <= B(d - mid - 1)) lo = mid + 1;
        else hi = mid;
      }
      uint32_t ia = lo, ib = d - lo;
      const uint32_t e = d + per < lq ? d + per : lq;
      for (uint32_t o = d; o < e; ++o) {
        const bool take_a = ib >= np || (ia < mm && A(ia) <= B(ib));
        Q[o] = take_a ? A(ia) : B(ib);
        if (!take_a) atomicOr(&h.pkg[j - 1][o >> 5], 1u << (o & 31));
        ia += take_a ? 1 : 0;
        ib += take_a ? 0 : 1;
      }
    }
    wsync();
    lp = lq;
  }
  // selection, top level down (lane 0; 15 steps of a popcount)
  if (lane == 0) {
    uint32_t c = cap;
    for (int j = limit - 1; j >= 1; --j) {
      uint32_t pk = 0;
      for (uint32_t w = 0; w < (c >> 5); ++w) pk += __popc(h.pkg[j - 1][w]);
      if (c & 31) pk += __popc(h.pkg[j - 1][c >> 5] & ((1u << (c & 31)) - 1));
      h.items[j] = c - pk;
      c = 2 * pk;
    }
    h.items[0] = c;
  }
  wsync();
  for (uint32_t k = lane; k < mm; k += 64) {
    uint32_t l = 0;
    for (int j = 0; j < limit; ++j) l += k < h.items[j] ? 1u : 0u;
    len_out[h.key[k] & 511] = (uint8_t)l;
  }
  wsync();
}

// canonical codes (bit-reversed for LSB-first emission), wave-parallel: the
// rank of a symbol among equal lengths by ballots per 64-symbol chunk
__device__ void huff_codes(const uint8_t *len, int n, uint32_t *code) {
  const int lane = threadIdx.x & 63;
  uint32_t cnt = 0;  // lane l < 16: symbols of length l
  for (int b0 = 0; b0 < n; b0 += 64) {
    const int i = b0 + lane;
    const uint32_t l = i < n ? len[i] : 0u;
#pragma unroll
    for (int L = 1; L < 16; ++L) {
      const uint32_t c = (uint32_t)__popcll(__ballot(l == (uint32_t)L));
      if (lane == L) cnt += c;
    }
  }
  // first code of each length: next[l] = (next[l-1] + cnt[l-1]) << 1
  uint32_t next = 0, run = 0;
  for (int L = 1; L < 16; ++L) {
    const uint32_t prev_cnt = L > 1 ? (uint32_t)__builtin_amdgcn_readlane((int)cnt, L - 1) : 0u;
    run = (run + prev_cnt) << 1;
    if (lane == L) next = run;
  }
  for (int b0 = 0; b0 < n; b0 += 64) {
    const int i = b0 + lane;
    const uint32_t l = i < n ? len[i] : 0u;
    uint32_t v = 0;
#pragma unroll
    for (int L = 1; L < 16; ++L) {
      const uint64_t peers = __ballot(l == (uint32_t)L);
      const uint32_t base = (uint32_t)__builtin_amdgcn_readlane((int)next, L);
      if (l == (uint32_t)L) v = base + (uint32_t)__popcll(peers & lanemask_lt(lane));
      if (lane == L) next += (uint32_t)__popcll(peers);
    }
    if (i < n) code[i] = l ? ((l << 16) | (__brev(v) >> (32 - l))) : 0u;
  }
  wsync();
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


// LDS histogram increment as inline asm: the compiler puts an
// s_waitcnt vmcnt(0) before every LDS store it sees while LDS-DMA loads are in
// flight (it cannot tell the parse ring from the histograms), which would
// drain parse_block_dma's prefetch at every window.  (LDS operations complete
// in order, so the compiler's own lgkmcnt waits stay sufficient.)
__device__ __forceinline__ void lds_inc(uint32_t *p) {
  const uint32_t a = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint32_t *)p;
  __asm__ volatile("ds_add_u32 %0, %1" ::"v"(a), "v"(1u) : "memory");
}

#ifndef ZT_PW_SCALAR
#define ZT_PW_SCALAR 3  // match lanes up to which a window's path is walked by scalar jumps
#endif
// parse -> tokens over res, histograms.  One 64-position window per step:
// the path through it from `entry` (a scalar walk over the match lanes, or
// pointer doubling when they are many), its tokens written in order.
// (WRITE = false: histograms of the greedy parse only, res untouched)
template <bool WRITE, class S>
__device__ __forceinline__ void parse_window(S *s, const DeflateParams &P, uint32_t *r_blk, uint32_t len, uint32_t w0,
                                             uint32_t r, uint32_t r_next, uint32_t &entry, uint32_t &ntok) {
  const int lane = threadIdx.x & 63;
    const uint32_t i = w0 + lane;
    uint32_t L = res_len(r);
    if (P.lazy && !P.opt) {
      // one-step lazy: a longer match at i + 1 defers this one
      uint32_t nb = res_len((uint32_t)__shfl_down((int)r, 1, 64));
      const uint32_t first_next = res_len((uint32_t)__shfl((int)r_next, 0, 64));
      if (lane == 63) nb = first_next;
      if (L >= 3 && i + 1 < len && nb > L) L = 0;
    }
    // the path through the window.  Few match lanes past the entry: a scalar
    // walk (literal runs up to the next match lane, then a jump past it);
    // many: pointer doubling (6 rounds of lane shuffles)
    const uint64_t valid = __ballot(i < len);
    const uint64_t mm = __ballot(i < len && L >= 3);
    uint64_t path = 0;
    uint32_t exit;
    if (__popcll(mm & (~0ull << entry)) <= ZT_PW_SCALAR) {
      uint32_t cur = entry;
      while (cur < 64) {
        const uint64_t rest = mm & (~0ull << cur);
        const uint32_t m = rest ? (uint32_t)__builtin_ctzll(rest) : 64u;
        path |= (m >= 64 ? ~0ull : ((1ull << m) - 1)) & (~0ull << cur);
        if (m >= 64) {
          cur = 64;
          break;
        }
        path |= 1ull << m;
        cur = m + (uint32_t)__builtin_amdgcn_readlane((int)L, (int)m);
      }
      path &= valid;
      exit = cur;
    } else {
      const uint32_t step = L >= 3 ? L : 1;
      uint32_t ptr = i < len ? lane + step : 64u;
      uint64_t mask = i < len ? 1ull << lane : 0ull;
      // rounds until every lane's chain has left the window (at most 6)
      for (int rnd = 0; rnd < 6 && __ballot(ptr < 64); ++rnd) {
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
      path = ((uint64_t)path_hi << 32) | path_lo;
      exit = (uint32_t)__builtin_amdgcn_readlane((int)ptr, (int)entry);
    }
    const bool on = (path >> lane) & 1;
    // one literal / length increment for every path lane, then the distances
    // (the two branches issued one LDS atomic instruction each: parse 2.35 ->
    // 2.29 ms, price 0.565 -> 0.554 per GiB, streams identical, gpurun_out/abH)
    if (on) {
      const bool mt = L >= 3;
      const uint32_t token = mt ? (L << 16) | res_dist(r) : res_byte(r);
      lds_inc(&s->lit_hist[mt ? 257 + len_sym(L) : token]);
      if (mt) {
        uint32_t eb, ev;
        lds_inc(&s->dist_hist[dist_sym(res_dist(r), eb, ev)]);
      }
      if (WRITE) r_blk[ntok + __popcll(path & lanemask_lt(lane))] = token;
    }
    ntok += __popcll(path);
    entry = exit - 64;
}

// register-prefetch driver (any alignment / length)
constexpr int PB_PF = 6;  // parse windows prefetched
template <bool WRITE, class S>
__device__ uint32_t parse_block_regs(S *s, const DeflateParams &P, uint32_t *r_blk, uint32_t len) {
  const int lane = threadIdx.x & 63;
  uint32_t entry = 0;  // first path position relative to the current window
  uint32_t ntok = 0;
  // software pipeline: PB_PF windows' loads are in flight while one is parsed
  // (rq[j] holds window w0 + 64 j; rq[j + 1] is the lazy look-ahead)
  uint32_t rq[PB_PF];
#pragma unroll
  for (int j = 0; j < PB_PF; ++j) {
    const uint32_t p = 64u * j + lane;
    rq[j] = p < len ? r_blk[p] : 0u;
  }
  for (uint32_t wb = 0; wb < len; wb += 64 * PB_PF) {
#pragma unroll
    for (int j = 0; j < PB_PF; ++j) {
      const uint32_t w0 = wb + 64u * j;
      if (w0 >= len) break;
      const uint32_t r = rq[j];
      {
        const uint32_t p = w0 + 64u * PB_PF + lane;
        rq[j] = p < len ? r_blk[p] : 0u;
      }
      const uint32_t r_next = rq[(j + 1) % PB_PF];
      if (entry >= 64) {
        entry -= 64;
        continue;
      }
      parse_window<WRITE>(s, P, r_blk, len, w0, r, r_next, entry, ntok);
    }
  }
  return ntok;
}

// LDS-DMA driver for whole, 4-byte aligned blocks: chunks of PB_CH windows
// (res words and data bytes) stream into a ring of PB_NCH chunks by
// global_load_lds, PB_NCH - 1 chunks ahead, with one counted vmcnt wait per
// chunk -- the register driver's loads could not stay in flight across the
// window loop's branches (the compiler waited for each window's loads).
__device__ __forceinline__ void vm_wait_loads(void) {
  // vmcnt(PB_LOADS * (PB_NCH - 2)): chunks c and c + 1 have landed (loads
  // complete in order; stores in between only make this wait longer)
  constexpr int N = PB_LOADS * (PB_NCH - 2);
  static_assert(N < 64, "vmcnt field");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | 0x0F70);
}
template <bool WRITE, class S>
__device__ uint32_t parse_block_dma(S *s, ParseStage *st, const DeflateParams &P, uint32_t *r_blk, uint32_t len) {
  const int lane = threadIdx.x & 63;
  const uint32_t nch = len / (PB_CH * 64);  // len: a multiple of PB_CH * 64
  auto issue = [&](uint32_t c) {
    // past the block: re-read chunk 0 (the count of loads stays fixed)
    const uint32_t cc = c < nch ? c : 0u;
    const uint32_t slot = c % PB_NCH;
#pragma unroll
    for (int w = 0; w < PB_CH; ++w)
      __builtin_amdgcn_global_load_lds(r_blk + cc * (PB_CH * 64) + w * 64 + lane, &st->res[slot][w * 64], 4, 0, 0);
  };
#pragma unroll
  for (int c = 0; c < PB_NCH - 1; ++c) issue((uint32_t)c);
  uint32_t entry = 0, ntok = 0;
  for (uint32_t c = 0; c < nch; ++c) {
    issue(c + PB_NCH - 1);
    vm_wait_loads();
    const uint32_t slot = c % PB_NCH, nslot = (c + 1) % PB_NCH;
    for (int w = 0; w < PB_CH; ++w) {
      const uint32_t w0 = c * (PB_CH * 64) + (uint32_t)w * 64;
      if (entry >= 64) {
        entry -= 64;
        continue;
      }
      const uint32_t r = st->res[slot][w * 64 + lane];
      const uint32_t r_next = w + 1 < PB_CH ? st->res[slot][(w + 1) * 64] : st->res[nslot][0];
      parse_window<WRITE>(s, P, r_blk, len, w0, r, r_next, entry, ntok);
    }
  }
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): no DMA into the ring after return
  return ntok;
}

template <bool WRITE, class S>
__device__ uint32_t parse_block(S *s, ParseStage *st, const DeflateParams &P, uint32_t *r_blk, uint32_t len) {
  if (len % (PB_CH * 64) == 0 && len > 0) return parse_block_dma<WRITE>(s, st, P, r_blk, len);
  return parse_block_regs<WRITE>(s, P, r_blk, len);
}

// ================================ 1b. optparse_kernel ================================
// Cost-based parse of one 32 KiB block per wavefront (levels with opt = 1).
// price_kernel: the greedy parse of the block gives symbol statistics; their
// entropy gives a price per literal, length and distance symbol (1/8 bit
// units, <= 15 bits per symbol).  optparse_kernel: each lane runs a backward
// shortest-path DP over its own 512-position segment (plus OP_OV = 64
// positions of the next segment, where paths have converged): C[i] =
// min(lit(i) + C[i+1], min_l len(l) + dist(D_i) + C[i+l]) over l in
// 3..min(L_i, OP_SHORT) and l = L_i, for the longest match
// (L_i, D_i) the match kernel found at i.  The chosen length is written over
// res[i] (0 = literal), so the block kernel's parse follows the DP's path.
// Every value left in res is a valid (shorter or equal) match, so the stream
// stays correct whatever the cost model says.
// C is kept modulo 2^16 in an OP_RING-row LDS ring per lane (row = step mod OP_RING,
// all lanes on the same row at the same step, so reads of one length l hit
// distinct banks): differences over <= 258 positions stay below 2^15.
typedef unsigned int op_u32x4 __attribute__((ext_vector_type(4)));
constexpr int OP_SEG = DF_BLOCK / 64;  // one segment per lane
#ifndef ZT_OP_OV
#define ZT_OP_OV 64  // 128 / 96 / 64 / 32: post-match 7.64 / 7.50 / 7.42 / 7.28 ms per GiB, worst ratio window 1.0179 / 1.0180 / 1.0182 / 1.0195 (tools/gpu_r04ov.sh)
#endif
constexpr int OP_OV = ZT_OP_OV;  // positions of the next segment each lane's DP runs over (paths converge)
// C ring rows: C[i + l] for l <= OP_RING.  A longer match reads C[i + OP_RING]
// instead of C[i + L] (an estimate of its continuation: the parse stays
// valid, only the DP's cost model is approximate there); 64 rows keep the
// LDS at 8.5 KiB (round 2, 16-position groups: 80 rows / 4 groups, 3 waves
// per SIMD, 2.83 ms against 2.73 at 64 / 3 and 4 waves,
// profiles/r02q_optparse_variants.txt; bench ratio unchanged to 5 digits;
// 260 rows: 1 wave per SIMD)
#ifndef ZT_OP_RING
#define ZT_OP_RING 64
#endif
constexpr int OP_RING = ZT_OP_RING;
#ifndef ZT_OP_SHORT
#define ZT_OP_SHORT 24  // 8..14 / 16 / 18 / 20: worst ratio window 1.042..1.026 / 1.0182 / 1.0153 / 1.0144 at chain 28; at chain 20: 20 / 24 / 28 1.0207 / 1.0190 / 1.0188 -- the headroom spent on level 6's chain 28 -> 20 (profiles/r04os_sweep.txt)
#endif
constexpr int OP_SHORT = ZT_OP_SHORT;  // every cut length 3..OP_SHORT is tried (even), longer ones only at L
static_assert(OP_SHORT % 2 == 0 && OP_SHORT >= 4, "cut lengths go in pairs");
#ifndef ZT_OP_PF
#define ZT_OP_PF 1
#endif
constexpr int OP_PF = ZT_OP_PF;
constexpr int OP_G = 32;  // positions per group (one 128-byte line of res)

// prices of one block, in 1/8 bits (price_kernel -> optparse_kernel), kept at
// the start of the block's slot until block_kernel writes its header there
struct BlockPrices {
  uint8_t litc[256];
  uint8_t lenc[260];  // by match length (3..258), extra bits included
  uint8_t distc[32];  // by distance symbol, extra bits included
  uint32_t any_match;
};

struct PriceShared {
  uint32_t lit_hist[288];
  uint32_t dist_hist[32];
  ParseStage stage;
};

__device__ __forceinline__ uint32_t op_price(uint32_t f, float inv_total) {
  // -log2((f + 0.5) / total) in 1/8 bits, clamped to [1, 15] bits
  float b = -__log2f(((float)f + 0.5f) * inv_total) * 8.0f;
  int c = (int)(b + 0.5f);
  return (uint32_t)(c < 8 ? 8 : c > 120 ? 120 : c);
}

// price sample: 1/ZT_PRICE_SAMPLE of each block in ZT_PRICE_PIECES pieces
// spread over it.  The block's first 1/4 (sample 4, one piece) -> 1/8 in eight
// 512-position pieces: price 0.55 -> 0.30 ms per GiB, streams smaller at
// levels 6 and 9 (bench corpus at 128 MiB 0.53382 -> 0.53379), gate worst
// 1.0193 -> 1.0191.  1/4 in 4 pieces: price unchanged, gate 1.0193; 1/8 in 4:
// 0.29 ms, 1.0192; 1/16 in 4: 0.16 ms, 1.0197 (gpurun_out/abS4, abS8, abC,
// abS16, abS8p8)
#ifndef ZT_PRICE_SAMPLE
#define ZT_PRICE_SAMPLE 8
#endif
#ifndef ZT_PRICE_PIECES
#define ZT_PRICE_PIECES 8
#endif
// greedy parse statistics -> prices (one wave per block, small LDS: many waves per CU)
__global__ __launch_bounds__(64) void price_kernel(DeflateParams P) {
  __shared__ PriceShared sh;
  PriceShared *s = &sh;
  const int lane = threadIdx.x;
  const uint32_t blk = blockIdx.x;
  if (P.store && P.store[blk]) return;  // stored block (classify_kernel)
  const uint64_t lo = (uint64_t)blk * DF_BLOCK;
  const uint64_t n = stream_end(P, blk);
  const uint32_t blen = (uint32_t)((n - lo) < DF_BLOCK ? (n - lo) : DF_BLOCK);
  for (int i = lane; i < 288; i += 64) s->lit_hist[i] = 0;
  if (lane < 32) s->dist_hist[lane] = 0;
  wsync();
  // the prices only need symbol statistics: a greedy parse of 1/ZT_PRICE_SAMPLE
  // of the block estimates them (a short block: its start, or all of it)
  const uint32_t plen = blen < (uint32_t)(DF_BLOCK / ZT_PRICE_SAMPLE) ? blen : (uint32_t)(DF_BLOCK / ZT_PRICE_SAMPLE);
  if (ZT_PRICE_PIECES > 1 && blen == DF_BLOCK) {
    // the sample in ZT_PRICE_PIECES pieces spread over the block, each parsed
    // greedily from its own start
    constexpr uint32_t pl = DF_BLOCK / ZT_PRICE_SAMPLE / ZT_PRICE_PIECES;
    static_assert(pl % (PB_CH * 64) == 0, "pieces take the LDS-DMA driver");
    for (int j = 0; j < ZT_PRICE_PIECES; ++j)
      parse_block<false>(s, &s->stage, P, P.res + lo + (uint64_t)j * (DF_BLOCK / ZT_PRICE_PIECES), pl);
  } else {
    parse_block<false>(s, &s->stage, P, P.res + lo, plen);
  }
  wsync();
  BlockPrices *bp = reinterpret_cast<BlockPrices *>(P.slots + (size_t)blk * DF_SLOT);
  float tl = 0.f, td = 0.f;
  for (int i = lane; i < 286; i += 64) tl += (float)s->lit_hist[i] + 0.5f;
  uint32_t dsum = lane < 30 ? s->dist_hist[lane] : 0u;
  if (lane < 30) td = (float)dsum + 0.5f;
  for (int off = 32; off; off >>= 1) {
    tl += __shfl_xor(tl, off, 64);
    td += __shfl_xor(td, off, 64);
    dsum += __shfl_xor(dsum, off, 64);
  }
  const float il = 1.0f / tl, id = 1.0f / td;
  for (int i = lane; i < 256; i += 64) bp->litc[i] = (uint8_t)op_price(s->lit_hist[i], il);
  if (lane < 32) bp->distc[lane] = lane < 30 ? (uint8_t)(op_price(s->dist_hist[lane], id) + 8 * dist_extra(lane)) : 255;
  for (int l = lane; l < 260; l += 64) {
    uint8_t v = 255;
    if (l >= 3 && l <= 258) {
      const uint32_t ls = len_sym(l);
      v = (uint8_t)(op_price(s->lit_hist[257 + ls], il) + 8 * len_extra(ls));
    }
    bp->lenc[l] = v;
  }
  if (lane == 0) bp->any_match = dsum;
}

struct OptShared {
  BlockPrices pr;
  uint16_t ring[OP_RING][64];
};

__device__ __forceinline__ uint32_t op_min3(uint32_t a, uint32_t b, uint32_t c) {
  uint32_t r;
  asm("v_min3_u32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}

#ifndef ZT_OP_MINW
#define ZT_OP_MINW 3  // waves per SIMD the register budget must allow (168 VGPRs: cut lengths to 24 take 138; at 4 waves, 128 VGPRs, 20 and more spill: optparse +0.1 ms)
#endif
__global__ __launch_bounds__(64, ZT_OP_MINW) void optparse_kernel(DeflateParams P) {
  __shared__ OptShared sh;
  OptShared *s = &sh;
  const int lane = threadIdx.x;
  const uint32_t blk = blockIdx.x;
  if (P.store && P.store[blk]) return;  // stored block (classify_kernel)
  const uint64_t lo = (uint64_t)blk * DF_BLOCK;
  const uint64_t n = stream_end(P, blk);
  const uint32_t blen = (uint32_t)((n - lo) < DF_BLOCK ? (n - lo) : DF_BLOCK);
  uint32_t *r_blk = P.res + lo;
  const BlockPrices *bp = reinterpret_cast<const BlockPrices *>(P.slots + (size_t)blk * DF_SLOT);
  if (bp->any_match == 0) return;  // no match anywhere: the greedy parse is all literals already
  {
    const uint32_t *src = reinterpret_cast<const uint32_t *>(bp);
    uint32_t *dst = reinterpret_cast<uint32_t *>(&s->pr);
    for (int i = lane; i < (int)(sizeof(BlockPrices) / 4); i += 64) dst[i] = src[i];
    uint32_t *rw = reinterpret_cast<uint32_t *>(&s->ring[0][0]);
    for (int i = lane; i < OP_RING * 32; i += 64) rw[i] = 0;
  }
  wsync();
  uint32_t lk[OP_SHORT + 1];  // price << 9 | l of the cut lengths (wave-uniform, SGPRs)
#pragma unroll
  for (int l = 3; l <= OP_SHORT; ++l)
    lk[l] = (uint32_t)__builtin_amdgcn_readfirstlane((int)(((uint32_t)s->pr.lenc[l] << 9) | (uint32_t)l));
  // backward DP, one segment per lane
  const uint32_t s0 = (uint32_t)lane * OP_SEG;
  if (s0 < blen) {
    const uint32_t seg_end = s0 + OP_SEG < blen ? s0 + OP_SEG : blen;
    const uint32_t e = seg_end + OP_OV < blen ? seg_end + OP_OV : blen;
    uint32_t C1 = 0;   // C[i + 1]
    uint32_t row = 0;  // step mod OP_RING
    uint32_t cr9[OP_SHORT + 1];  // cr9[l] = C[i + l] << 9 (0 past the segment's end)
#pragma unroll
    for (int l = 0; l <= OP_SHORT; ++l) cr9[l] = 0;
    const uint32_t g_last = (e - 1) & ~uint32_t(OP_G - 1);
    const uint32_t ngroups = (g_last - s0) / OP_G + 1;
    // a group is OP_G = 32 positions: one whole 128-byte line of res per
    // lane (the literal's byte rides in res), so the 64 lanes' scattered
    // reads each use the full line they fetch (16-position groups read half
    // lines + 16 data bytes: 13.4 GB of reads per GiB, profiles/r04pmc_*)
    auto load_g = [&](uint32_t g, op_u32x4 *r4) {
      const op_u32x4 *src = reinterpret_cast<const op_u32x4 *>(r_blk + g);
#pragma unroll
      for (int q = 0; q < OP_G / 4; ++q) r4[q] = src[q];
    };
    // OP_PF groups in flight per lane: HBM latency is hidden by depth
    op_u32x4 rq[OP_PF][OP_G / 4];
#pragma unroll
    for (int j = 0; j < OP_PF; ++j)
      if ((uint32_t)j < ngroups) load_g(g_last - (uint32_t)OP_G * (uint32_t)j, rq[j]);
    uint32_t gi = 0;  // groups done
    while (gi < ngroups) {
#pragma unroll
      for (int j = 0; j < OP_PF; ++j) {
        if (gi < ngroups) {
          const uint32_t g = g_last - (uint32_t)OP_G * gi;
          op_u32x4 rv[OP_G / 4];
#pragma unroll
          for (int q = 0; q < OP_G / 4; ++q) rv[q] = rq[j][q];
          if (gi + OP_PF < ngroups) load_g(g - (uint32_t)OP_G * OP_PF, rq[j]);
#pragma unroll
          for (int k = OP_G - 1; k >= 0; --k) {
            // positions >= e (the tail of the block's last group) are steps
            // with price 0 and no match: C stays 0 there, as past the end
            const uint32_t i = g + (uint32_t)k;
            const bool live = i < e;
            {
              const uint32_t r = rv[k >> 2][k & 3];
              const uint32_t L = live ? res_len(r) : 0u, D = res_dist(r);
              // C[i+1 .. i+OP_SHORT] live in registers (cr[1..]); only the
              // full-length candidate reads the LDS ring.  Candidates are
              // compared as keys (price relative to C[i+1], biased) << 9 | l.
              uint32_t eb, ev;
              const uint32_t Dc = D ? D : 1u;
              const int dc = (int)s->pr.distc[dist_sym(Dc, eb, ev)];
              const uint32_t Lc = L < 3 ? 3u : L;
              const uint32_t Lr = Lc < (uint32_t)OP_RING ? Lc : (uint32_t)OP_RING;
              const uint32_t rr = row >= Lr ? row - Lr : row + OP_RING - Lr;
              const int c_far = (int)(int16_t)(uint16_t)(s->ring[rr][lane] - (uint16_t)C1) + (int)s->pr.lenc[Lc];
              const int lit = live ? (int)s->pr.litc[res_byte(r)] : 0;
              uint32_t key = (uint32_t)(lit + 0x8000) << 9;
              // key of length l: (price + C[i+l] - C[i+1] + bias) << 9 | l,
              // one add3 of pre-shifted terms (exact modulo 2^32: the
              // unshifted value is below 2^23)
              const uint32_t base9 = (uint32_t)(dc + 0x8000 - (int)C1) << 9;
              // a pair of cut lengths enters when both are valid (one compare
              // and one select per pair: optparse 2.63 -> 2.41 ms per GiB with
              // two selects under one compare, r05au); the odd length L
              // itself, whose pair does not, is the full-length candidate
              // below, taken for every match (the same key: C[i + L] from the
              // ring)
#pragma unroll
              for (uint32_t l = 3; l < OP_SHORT; l += 2) {
                const uint32_t ka = base9 + cr9[l] + lk[l], kb = base9 + cr9[l + 1] + lk[l + 1];
                const uint32_t m = op_min3(key, ka, kb);
                key = l + 1 <= L ? m : key;
              }
              {
                const uint32_t kl = ((uint32_t)(dc + 0x8000 + c_far) << 9) | (Lc & 511);
                key = (L >= 3 && kl < key) ? kl : key;
              }
              const uint32_t choice = key & 511;
              const int best = (int)(key >> 9) - 0x8000;
              C1 += (uint32_t)best;
              s->ring[row][lane] = (uint16_t)C1;
              row = row + 1 == OP_RING ? 0 : row + 1;
#pragma unroll
              for (int l = OP_SHORT; l > 1; --l) cr9[l] = cr9[l - 1];
              cr9[1] = C1 << 9;
              rv[k >> 2][k & 3] = (r & 0xFF000000u) | (choice << 15) | D;
            }
          }
          // the group's choices in whole-line stores (positions >= seg_end
          // belong to the next lane; a group straddles seg_end only at the
          // block's end, where the positions past blen are never read)
          if (g < seg_end) {
            op_u32x4 *dst = reinterpret_cast<op_u32x4 *>(r_blk + g);
#pragma unroll
            for (int q = 0; q < OP_G / 4; ++q) dst[q] = rv[q];
          }
          ++gi;
        }
      }
    }
  }
}

// parse of one block per wave (the DP's path, or the greedy / lazy parse):
// tokens written over res, literal / length and distance histograms and the
// token count handed to block_kernel through the start of the block's slot
// (its prices are consumed by then; block_kernel writes the header there only
// after reading them).  A kernel of its own so that its LDS (histograms + the
// LDS-DMA staging ring, 7.5 KiB) keeps 20 waves per CU on this latency-bound
// walk, instead of block_kernel's 15 (its Huffman scratch, 10.3 KiB).
__global__ __launch_bounds__(64) void parse_kernel(DeflateParams P) {
  __shared__ PriceShared sh;
  PriceShared *s = &sh;
  const int lane = threadIdx.x;
  const uint32_t blk = blockIdx.x;
  if (P.store && P.store[blk]) return;  // stored block (classify_kernel)
  const uint64_t lo = (uint64_t)blk * DF_BLOCK;
  const uint64_t n = stream_end(P, blk);
  const uint32_t blen = (uint32_t)((n - lo) < DF_BLOCK ? (n - lo) : DF_BLOCK);
  for (int i = lane; i < 288; i += 64) s->lit_hist[i] = 0;
  if (lane < 32) s->dist_hist[lane] = 0;
  wsync();
  const uint32_t ntok = parse_block<true>(s, &s->stage, P, P.res + lo, blen);
  wsync();
  uint32_t *hs = reinterpret_cast<uint32_t *>(P.slots + (size_t)blk * DF_SLOT);
  for (int i = lane; i < 288; i += 64) hs[i] = s->lit_hist[i];
  if (lane < 32) hs[288 + lane] = s->dist_hist[lane];
  if (lane == 0) hs[320] = ntok;
}

// one wave per DEFLATE block: launched per parse block, the group's leader
// works, the others return
__global__ __launch_bounds__(64) void block_kernel(DeflateParams P) {
  __shared__ BlockShared sh;
  BlockShared *s = &sh;
  const int lane = threadIdx.x;
  const uint32_t blk = blockIdx.x;
  if (!group_leader(P, blk)) return;
  const uint32_t nsub = group_size(P, blk);
  const uint64_t lo = (uint64_t)blk * DF_BLOCK;
  const uint64_t n = stream_end(P, blk);
  const uint64_t gspan = (uint64_t)nsub * DF_BLOCK;
  const uint32_t blen = (uint32_t)((n - lo) < gspan ? (n - lo) : gspan);
  BlockPlan *plan = P.plans + blk;
  const bool last = P.span ? lo + gspan >= n : P.final_ && (blk + nsub == P.nblocks);
  if (P.store && P.store[blk]) {  // classify_kernel: bytes that cannot beat a stored block
    if (lane == 0) P.slot_len[blk] = blen + 5 * ((blen + 65534) / 65535) + 5;
    if (lane > 0 && (uint32_t)lane < nsub) P.slot_len[blk + lane] = 0;
    if (lane == 0) {
      plan->ntok = 0;
      plan->btype = 0;
      plan->hdr_bits = 0;
      plan->hdr_tail = 0;
      plan->blen = blen;
      plan->last = last ? 1 : 0;
      plan->nsub = nsub;
    }
    return;
  }
  // the parse's histograms and token counts (parse_kernel, in each parse
  // block's slot), summed over the group
  uint32_t ntok = 0;
  for (uint32_t k = 0; k < nsub; ++k) {
    const uint32_t *hs = reinterpret_cast<const uint32_t *>(P.slots + (size_t)(blk + k) * DF_SLOT);
    for (int i = lane; i < 288; i += 64) s->lit_hist[i] = (k ? s->lit_hist[i] : 0u) + hs[i];
    if (lane < 32) s->dist_hist[lane] = (k ? s->dist_hist[lane] : 0u) + hs[288 + lane];
    const uint32_t nt = hs[320];
    if (lane == 0) plan->ntok_sub[k] = nt;
    ntok += nt;
  }
  wsync();
#ifdef ZT_DF_TIME
  uint64_t bt0 = __builtin_readcyclecounter(), btk;
#define BK_T(k)                                                                          \
  btk = __builtin_readcyclecounter();                                                    \
  if (lane == 0) atomicAdd(&g_bk_time[k], (unsigned long long)(btk - bt0));              \
  bt0 = btk;
#else
#define BK_T(k) (void)0
#endif
  BK_T(0);
  wsync();
  if (lane == 0) s->lit_hist[256] += 1;  // end of block
  wsync();
  huff_lengths(s, s->lit_hist, 286, 15, s->lit_len);
  huff_lengths(s, s->dist_hist, 30, 15, s->dist_len);
  BK_T(1);
  {
    // trailing zero lengths trimmed (RFC 1951 3.2.7: HLIT >= 257, HDIST >= 1)
    uint32_t hi_lit = 0;
    for (int c = 0; c < 5; ++c) {
      const int i = c * 64 + lane;
      const uint64_t nz = __ballot(i < 286 && s->lit_len[i] != 0);
      if (nz) hi_lit = (uint32_t)(c * 64 + 64 - __clzll(nz));
    }
    const uint64_t dnz = __ballot(lane < 30 && s->dist_len[lane] != 0);
    const uint32_t hlit = hi_lit > 257 ? hi_lit : 257;
    const uint32_t hdist = dnz ? (uint32_t)(64 - __clzll(dnz)) : 1u;
    const uint32_t total = hlit + hdist;
    if (lane < 19) s->cl_code[lane] = 0;  // CL symbol frequencies until the codes are built
    if (lane == 0) {
      s->hlit = hlit;
      s->hdist = hdist;
    }
    wsync();
    // RLE of the concatenated lengths, one lane per run: runs start where the
    // value changes; each run's symbols are counted, placed by a scan, then
    // written by its lane
    auto val = [&](uint32_t i) -> uint32_t { return i < hlit ? s->lit_len[i] : s->dist_len[i - hlit]; };
    uint64_t starts[5];
    for (int c = 0; c < 5; ++c) {
      const uint32_t i = (uint32_t)(c * 64 + lane);
      starts[c] = __ballot(i < total && (i == 0 || val(i) != val(i - 1)));
    }
    uint32_t base = 0;
    for (int c = 0; c < 5; ++c) {
      const uint32_t i = (uint32_t)(c * 64 + lane);
      const bool st = (starts[c] >> lane) & 1;
      uint32_t v = 0, r = 0, cnt = 0;
      if (st) {
        // the run's end: the next start (or the end of the lengths)
        uint32_t e = total;
        const uint64_t rest = lane < 63 ? starts[c] & (~0ull << (lane + 1)) : 0ull;
        if (rest) {
          e = (uint32_t)(c * 64) + (uint32_t)__builtin_ctzll(rest);
        } else {
          for (int cc = c + 1; cc < 5; ++cc)
            if (starts[cc]) {
              e = (uint32_t)(cc * 64) + (uint32_t)__builtin_ctzll(starts[cc]);
              break;
            }
        }
        v = val(i);
        r = e - i;
        // symbol count of the run (the writer below, counting only)
        uint32_t q = r;
        if (v == 0) {
          while (q >= 11) {
            q -= q < 138 ? q : 138;
            ++cnt;
          }
          cnt += q >= 3 ? 1 : q;
        } else {
          cnt = 1;
          --q;
          while (q >= 3) {
            q -= q < 6 ? q : 6;
            ++cnt;
          }
          cnt += q;
        }
      }
      // exclusive scan of the counts
      uint32_t incl = cnt;
      for (int off = 1; off < 64; off <<= 1) {
        const uint32_t y = (uint32_t)__shfl_up((int)incl, off, 64);
        if (lane >= off) incl += y;
      }
      uint32_t o = base + incl - cnt;
      base += (uint32_t)__shfl((int)incl, 63, 64);
      if (st) {
        uint32_t q = r;
        if (v == 0) {
          while (q >= 11) {
            const uint32_t x = q < 138 ? q : 138;
            s->cl_syms[o++] = (uint16_t)(18 | ((x - 11) << 5));
            atomicAdd(&s->cl_code[18], 1u);
            q -= x;
          }
          if (q >= 3) {
            s->cl_syms[o++] = (uint16_t)(17 | ((q - 3) << 5));
            atomicAdd(&s->cl_code[17], 1u);
          } else if (q) {
            atomicAdd(&s->cl_code[0], q);
            for (; q; --q) s->cl_syms[o++] = 0;
          }
        } else {
          s->cl_syms[o++] = (uint16_t)v;
          uint32_t nv = 1;
          --q;
          while (q >= 3) {
            const uint32_t x = q < 6 ? q : 6;
            s->cl_syms[o++] = (uint16_t)(16 | ((x - 3) << 5));
            atomicAdd(&s->cl_code[16], 1u);
            q -= x;
          }
          for (; q; --q, ++nv) s->cl_syms[o++] = (uint16_t)v;
          atomicAdd(&s->cl_code[v], nv);
        }
      }
    }
    if (lane == 0) s->n_cl_syms = base;
  }
  wsync();
  BK_T(2);
  huff_lengths(s, s->cl_code, 19, 7, s->cl_len);
  huff_codes(s->lit_len, 286, s->lit_code);
  huff_codes(s->dist_len, 30, s->dist_code);
  huff_codes(s->cl_len, 19, s->cl_code);
  BK_T(3);
  // sizes of the three choices (bits, without the sync marker)
  uint64_t dyn = 0, fix = 0;
  for (int i = lane; i < 286; i += 64) {
    uint32_t f = s->lit_hist[i];
    uint32_t extra = i >= 257 ? len_extra(i - 257) : 0;
    dyn += (uint64_t)f * (s->lit_len[i] + extra);
    fix += (uint64_t)f * ((fixed_lit(i) >> 16) + extra);
  }
  if (lane < 30) {
    uint32_t f = s->dist_hist[lane];
    uint32_t extra = dist_extra(lane);
    dyn += (uint64_t)f * (s->dist_len[lane] + extra);
    fix += (uint64_t)f * (5 + extra);
  }
  uint32_t hclen = 19;
  while (hclen > 4 && s->cl_len[kClOrder[hclen - 1]] == 0) --hclen;
  uint32_t hdr = 0;
  for (uint32_t k = lane; k < s->n_cl_syms; k += 64) {
    uint32_t c = s->cl_syms[k] & 31;
    hdr += s->cl_len[c] + (c == 16 ? 2 : c == 17 ? 3 : c == 18 ? 7 : 0);
  }
  for (int off = 32; off; off >>= 1) {
    dyn += __shfl_xor(dyn, off, 64);
    fix += __shfl_xor(fix, off, 64);
    hdr += __shfl_xor(hdr, off, 64);
  }
  hdr += 3 + 5 + 5 + 4 + 3 * hclen;
  dyn += hdr;
  fix += 3;
  // stored: the block's bytes + 5 header bytes; Huffman forms add the
  // 3-bit marker header, padding and the 4 sync bytes
  const uint64_t stored_bits = 8ull * (blen + 5 * ((blen + 65534) / 65535) + 5);  // + its sync point
  const uint64_t dyn_bits = ((dyn + 3 + 7) & ~7ull) + 32;
  const uint64_t fix_bits = ((fix + 3 + 7) & ~7ull) + 32;
  BK_T(4);
  uint32_t bt;
  if (P.ctype == 1) bt = 1;
  else if (stored_bits <= dyn_bits && stored_bits <= fix_bits) bt = 0;
  else bt = dyn_bits <= fix_bits ? 2 : 1;
  // the block's exact size: scan_sizes places it before it is encoded
  if (lane == 0) P.slot_len[blk] = (uint32_t)((bt == 0 ? stored_bits : bt == 1 ? fix_bits : dyn_bits) >> 3);
  if (lane > 0 && (uint32_t)lane < nsub) P.slot_len[blk + lane] = 0;
  // codes for the encoder
  for (int i = lane; i < 288; i += 64) plan->lit_code[i] = bt == 2 ? (i < 286 ? s->lit_code[i] : 0u) : fixed_lit(i);
  if (lane < 32) plan->dist_code[lane] = bt == 2 ? (lane < 30 ? s->dist_code[lane] : 0u)
                                                 : ((5u << 16) | (__brev((uint32_t)lane) >> 27));
  // the dynamic header, wave-parallel: every field an item (value, bits),
  // bit offsets by a scan, OR-ed into an LDS word buffer (the package-merge
  // list space, free now), complete words copied to the slot
  uint32_t hbits = 0, htail = 0;
  if (bt == 1) {
    hbits = 3;
    htail = 2;  // BFINAL=0, BTYPE=01
  } else if (bt == 2) {
    uint32_t *hw = s->huf.lst[0];
    for (int k = lane; k < 160; k += 64) hw[k] = 0;
    wsync();
    const uint32_t nsym = s->n_cl_syms, nitems = 1 + hclen + nsym;
    uint32_t base = 0;
    for (uint32_t c0 = 0; c0 < nitems; c0 += 64) {
      const uint32_t it = c0 + (uint32_t)lane;
      uint32_t v = 0, nb = 0;
      if (it == 0) {
        v = 4u | ((s->hlit - 257) << 3) | ((s->hdist - 1) << 8) | ((hclen - 4) << 13);  // BTYPE=10, HLIT, HDIST, HCLEN
        nb = 17;
      } else if (it <= hclen) {
        v = s->cl_len[kClOrder[it - 1]];
        nb = 3;
      } else if (it < nitems) {
        const uint32_t cs = s->cl_syms[it - 1 - hclen], c = cs & 31;
        const uint32_t cc = s->cl_code[c], cl = cc >> 16;
        const uint32_t xb = c == 16 ? 2u : c == 17 ? 3u : c == 18 ? 7u : 0u;
        v = (cc & 0xFFFF) | ((cs >> 5) << cl);
        nb = cl + xb;
      }
      uint32_t incl = nb;
      for (int off = 1; off < 64; off <<= 1) {
        const uint32_t y = (uint32_t)__shfl_up((int)incl, off, 64);
        if (lane >= off) incl += y;
      }
      const uint32_t o = base + incl - nb;
      base += (uint32_t)__shfl((int)incl, 63, 64);
      if (nb) {
        const uint32_t sh = o & 31;
        atomicOr(&hw[o >> 5], v << sh);
        if (sh + nb > 32) atomicOr(&hw[(o >> 5) + 1], v >> (32 - sh));
      }
    }
    wsync();
    hbits = base;
    uint32_t *slot = reinterpret_cast<uint32_t *>(P.slots + (size_t)blk * DF_SLOT);
    for (uint32_t k = lane; k < (hbits >> 5); k += 64) slot[k] = hw[k];
    htail = hw[hbits >> 5] & ((hbits & 31) ? ((1u << (hbits & 31)) - 1) : 0u);
  }
  if (lane == 0) {
    plan->ntok = ntok;
    plan->btype = bt;
    plan->hdr_bits = hbits;
    plan->hdr_tail = htail;
    plan->blen = blen;
    plan->last = last ? 1 : 0;
    plan->nsub = nsub;
  }
  BK_T(5);
#ifdef ZT_DF_TIME
  if (lane == 0) atomicAdd(&g_bk_time[6], 1ull);
#endif
#undef BK_T
}

// ================================ 3. encode_kernel ================================
#ifndef ZT_ENC_LDS
#define ZT_ENC_LDS 1  // block words staged in LDS, then written out coalesced
#endif
#ifndef ZT_ENC_CACHE
#define ZT_ENC_CACHE (ZT_DF_GROUP == 1)  // a thread's first tokens kept in registers between the two passes
#endif
#ifndef ZT_ENC_NCACHE
#define ZT_ENC_NCACHE 32  // 16 / 32 / 48 / 64: encode 1.19 / 1.10 / 1.16 / 1.55 ms per GiB; L2 read requests 1.96 -> 1.16 GB (the second pass's re-reads missed L2; tools/gpu_r04ec*.sh)
#endif
constexpr int ENC_CACHE = ZT_ENC_NCACHE;  // tokens per thread kept (a multiple of 4)
// a dynamic block is never planned larger than its stored form
// (block_kernel); a fixed-code block (compressionType FIXED) may take 9 bits
// per byte: 36 KiB + header and marker
constexpr uint32_t ENC_OBUF_WORDS = (ZT_ENC_LDS ? (DF_GROUP * DF_BLOCK / 8 * 9 + 64) / 4 + 64 : 1);
struct EncShared {
  uint32_t lit_code[288];
  uint32_t dist_code[32];
  uint32_t start[ENC_THREADS + 1];  // exclusive prefix of per-thread bit counts
  uint32_t first_val[ENC_THREADS];  // contribution to the (partial) first word
  uint32_t wsum[ENC_THREADS / 64];
  uint32_t obuf[ENC_OBUF_WORDS];    // the block's words (ZT_ENC_LDS)
};

// a block's words in the stream: dst = the aligned word holding its first
// byte; words 0 and `wlast` are shared with the neighbouring blocks (or the
// restart marker), so only the block's own bytes [lo, hi) of them are stored.
// ZT_ENC_LDS: every word goes to the LDS buffer first -- each thread packs its
// own few words, so direct stores left most lines of the stream partially
// written per instruction (encode_kernel wrote 1.47 GB per GiB for 0.57 GB of
// stream, profiles/r04k_pmc_traffic.txt) -- and flush() writes them out
// coalesced.
struct BlockWords {
  uint8_t *dst;
  uint32_t wlast, lo, hi;
  uint32_t *obuf;
  __device__ __forceinline__ void store_global(uint32_t w, uint32_t v) const {
    if (w != 0 && w != wlast) {
      reinterpret_cast<uint32_t *>(dst)[w] = v;
      return;
    }
#pragma unroll
    for (uint32_t b = 0; b < 4; ++b) {
      const uint32_t x = 4 * w + b;
      if (x >= lo && x < hi) dst[x] = (uint8_t)(v >> (8 * b));
    }
  }
  __device__ __forceinline__ void store(uint32_t w, uint32_t v) const {
    if (ZT_ENC_LDS)
      obuf[w] = v;
    else
      store_global(w, v);
  }
  // after a workgroup barrier: words [0, wlast] from the LDS buffer
  __device__ __forceinline__ void flush(uint32_t t) const {
    if (!ZT_ENC_LDS) return;
    for (uint32_t w = t; w <= wlast; w += ENC_THREADS) store_global(w, obuf[w]);
  }
};

// bit accumulator writing aligned 32-bit words of one block
struct BitOut {
  uint64_t acc;
  uint32_t nacc;      // valid bits in acc (acc bit 0 = bit `word * 32` of the block's words)
  uint32_t word;      // index of the word acc starts at
  uint32_t first;     // first word index of this thread's range
  BlockWords slot;
  uint32_t first_val;
  bool first_partial;
  bool wrote_first;

  __device__ void init(uint32_t start_bit, const BlockWords &sl) {
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
        slot.store(word, w);
      }
      ++word;
      acc >>= 32;
      nacc -= 32;
    }
  }
};

__device__ __forceinline__ uint32_t token_bits(const EncShared *s, uint32_t tk) {
  if (tk < 256) return s->lit_code[tk] >> 16;
  const uint32_t L = tk >> 16, D = tk & 0xFFFF;
  const uint32_t ls = len_sym(L);
  uint32_t eb, ev;
  const uint32_t ds = dist_sym(D, eb, ev);
  return (s->lit_code[257 + ls] >> 16) + len_extra(ls) + (s->dist_code[ds] >> 16) + eb;
}

__device__ __forceinline__ void put_token(BitOut &bo, const EncShared *s, uint32_t tk) {
  if (tk < 256) {
    const uint32_t c = s->lit_code[tk];
    bo.put(c & 0xFFFF, c >> 16);
    return;
  }
  const uint32_t L = tk >> 16, D = tk & 0xFFFF;
  const uint32_t ls = len_sym(L);
  const uint32_t c = s->lit_code[257 + ls];
  bo.put(c & 0xFFFF, c >> 16);
  const uint32_t lx = len_extra(ls);
  if (lx) bo.put(L - len_base(ls), lx);
  uint32_t eb, ev;
  const uint32_t ds = dist_sym(D, eb, ev);
  const uint32_t dc = s->dist_code[ds];
  bo.put(dc & 0xFFFF, dc >> 16);
  if (eb) bo.put(ev, eb);
}

// f(token) for tokens [a, b) of this thread, read 64 bytes at a time (four
// 16-byte loads issued together): a thread's range is contiguous, so the
// lanes of a wave touch 64 different lines per load and one 4-byte load per
// token would fetch every line many times over
template <typename F>
__device__ __forceinline__ void for_tokens(const uint32_t *tok, uint32_t a, uint32_t b, F &&f) {
  typedef unsigned int u32x4t __attribute__((ext_vector_type(4)));
  uint32_t i = a;
  for (; i < b && (i & 3); ++i) f(tok[i]);
  for (; i + 16 <= b; i += 16) {
    const u32x4t *v = reinterpret_cast<const u32x4t *>(tok + i);
    const u32x4t x0 = v[0], x1 = v[1], x2 = v[2], x3 = v[3];
    f(x0.x); f(x0.y); f(x0.z); f(x0.w);
    f(x1.x); f(x1.y); f(x1.z); f(x1.w);
    f(x2.x); f(x2.y); f(x2.z); f(x2.w);
    f(x3.x); f(x3.y); f(x3.z); f(x3.w);
  }
  for (; i + 4 <= b; i += 4) {
    const u32x4t x = *reinterpret_cast<const u32x4t *>(tok + i);
    f(x.x); f(x.y); f(x.z); f(x.w);
  }
  for (; i < b; ++i) f(tok[i]);
}

// f(token) for tokens [a, b) of the group's concatenated token lists
template <typename F>
__device__ __forceinline__ void for_group_tokens(const DeflateParams &P, const BlockPlan *plan, uint32_t blk,
                                                 uint32_t a, uint32_t b, F &&f) {
  uint32_t off = 0;
  for (uint32_t k = 0; k < plan->nsub && off < b; ++k) {
    const uint32_t nk = plan->ntok_sub[k];
    const uint32_t lo = a > off ? a - off : 0u, hi = b - off < nk ? b - off : nk;
    if (lo < hi) for_tokens(P.res + (uint64_t)(blk + k) * DF_BLOCK, lo, hi, f);
    off += nk;
  }
}

// bytes [src, src + n) to [dst, dst + n) by the workgroup: dst-aligned words,
// each from two aligned source words (src may be unaligned)
__device__ __forceinline__ void enc_copy(uint8_t *dst, const uint8_t *src, uint32_t n, uint32_t t) {
  const uint32_t h0 = (4u - (uint32_t)((uintptr_t)dst & 3)) & 3, h = h0 < n ? h0 : n;
  if (t < h) dst[t] = src[t];
  const uint32_t n4 = (n - h) / 4;
  const uint8_t *s8 = src + h;
  uint32_t *d4 = reinterpret_cast<uint32_t *>(dst + h);
  const uint32_t sh = (uint32_t)((uintptr_t)s8 & 3);
  const uint32_t *s4 = reinterpret_cast<const uint32_t *>(s8 - sh);
  const uint32_t nsrc = (sh + 4 * n4 + 3) / 4;  // source words holding bytes of the copy
  for (uint32_t w = t; w < n4; w += ENC_THREADS) {
    const uint32_t lo = s4[w], hi = sh && w + 1 < nsrc ? s4[w + 1] : 0u;
    d4[w] = sh ? __builtin_amdgcn_alignbyte(hi, lo, sh) : lo;
  }
  for (uint32_t i = h + 4 * n4 + t; i < n; i += ENC_THREADS) dst[i] = src[i];
}

__device__ __forceinline__ bool restart_after(uint32_t b, uint32_t n, uint32_t restart, int final_,
                                              const uint64_t *span);
constexpr uint32_t kRestartMarkerLen = 10;

// one workgroup per DEFLATE block (launched per parse block; followers
// return): the block goes straight to its place in the stream, out +
// boff[blk] (its size was planned exactly by block_kernel and placed by
// scan_sizes), followed by the restart marker where a segment ends
__global__ __launch_bounds__(ENC_THREADS) void encode_kernel(DeflateParams P) {
  __shared__ EncShared sh;
  EncShared *s = &sh;
  const uint32_t t = threadIdx.x;
  const uint32_t blk = blockIdx.x;
  if (!group_leader(P, blk)) return;
  const BlockPlan *plan = P.plans + blk;
  const uint32_t bt = plan->btype, blen = plan->blen;
  const bool last = plan->last != 0;
  const uint8_t *slot_bytes = P.slots + (size_t)blk * DF_SLOT;
  uint8_t *dst = P.out + P.boff[blk];
  const uint32_t plan_bytes = P.slot_len[blk];
  if (t < kRestartMarkerLen && restart_after(blk + plan->nsub - 1, P.nblocks, P.restart, P.final_, P.span))
    dst[plan_bytes + t] = (t % 5) < 3 ? 0 : 0xFF;  // 00 00 00 FF FF x 2
  if (bt == 0) {
    // stored block: header byte, LEN, NLEN, data
    const uint8_t *raw = P.base + P.halo + (uint64_t)blk * DF_BLOCK;
    // followed, like every block, by an empty stored block (the sync point
    // inflate splits on), which carries BFINAL on the stream's last block
    // (pieces of at most 65535 bytes: a stored block's LEN is 16 bits)
    const uint32_t nparts = blen ? (blen + 65534) / 65535 : 1;
    if (t < nparts) {
      const uint32_t plen = blen - t * 65535 < 65535 ? blen - t * 65535 : 65535;
      uint8_t *h = dst + (size_t)t * (65535 + 5);
      h[0] = 0;
      h[1] = plen & 0xFF;
      h[2] = plen >> 8;
      h[3] = (~plen) & 0xFF;
      h[4] = ((~plen) >> 8) & 0xFF;
    }
    if (t == 0) {
      uint8_t *e = dst + 5 * nparts + blen;
      e[0] = last ? 1 : 0;
      e[1] = 0;
      e[2] = 0;
      e[3] = 0xFF;
      e[4] = 0xFF;
      if (blen + 5 * nparts + 5 != plan_bytes) atomicOr(P.fault, 1u);
    }
    for (uint32_t k = 0; k < nparts; ++k) {
      const uint32_t plen = blen - k * 65535 < 65535 ? blen - k * 65535 : 65535;
      enc_copy(dst + (size_t)k * (65535 + 5) + 5, raw + (size_t)k * 65535, plen, t);
    }
    return;
  }
  for (uint32_t i = t; i < 288; i += ENC_THREADS) s->lit_code[i] = plan->lit_code[i];
  if (t < 32) s->dist_code[t] = plan->dist_code[t];
  __syncthreads();
  const uint32_t ntok = plan->ntok;
  const uint32_t hdr_bits = plan->hdr_bits;
  const uint32_t a = (uint32_t)(((uint64_t)ntok * t) / ENC_THREADS);
  const uint32_t b = (uint32_t)(((uint64_t)ntok * (t + 1)) / ENC_THREADS);
  uint32_t bits = 0;
  const uint32_t *tok = P.res + (uint64_t)blk * DF_BLOCK;  // (DF_GROUP 1: the block's own tokens)
#if ZT_ENC_CACHE
  // the thread's first ENC_CACHE tokens stay in registers for the packing
  // pass (5 aligned 16-byte loads, then a shift by a % 4): only the rest is
  // read twice
  typedef unsigned int u32x4e __attribute__((ext_vector_type(4)));
  const uint32_t nc = b - a < (uint32_t)ENC_CACHE ? b - a : (uint32_t)ENC_CACHE;
  uint32_t cache[ENC_CACHE];
  {
    uint32_t raw[ENC_CACHE + 4];
    const u32x4e *v = reinterpret_cast<const u32x4e *>(tok + (a & ~3u));
#pragma unroll
    for (int q = 0; q < ENC_CACHE / 4 + 1; ++q) {
      const u32x4e x = (4 * q < (int)((a & 3) + nc)) ? v[q] : u32x4e{0, 0, 0, 0};
      raw[4 * q] = x.x;
      raw[4 * q + 1] = x.y;
      raw[4 * q + 2] = x.z;
      raw[4 * q + 3] = x.w;
    }
    const uint32_t sh = a & 3;
#pragma unroll
    for (int j = 0; j < ENC_CACHE; ++j)
      cache[j] = sh == 0 ? raw[j] : sh == 1 ? raw[j + 1] : sh == 2 ? raw[j + 2] : raw[j + 3];
  }
#pragma unroll
  for (int j = 0; j < ENC_CACHE; ++j)
    if ((uint32_t)j < nc) bits += token_bits(s, cache[j]);
  for_tokens(tok, a + nc, b, [&](uint32_t tk) { bits += token_bits(s, tk); });
#else
  if constexpr (DF_GROUP == 1)
    for_tokens(tok, a, b, [&](uint32_t tk) { bits += token_bits(s, tk); });
  else
    for_group_tokens(P, plan, blk, a, b, [&](uint32_t tk) { bits += token_bits(s, tk); });
#endif
  if (t == 0) bits += hdr_bits;
  const uint32_t eob = s->lit_code[256] >> 16;
  if (t == ENC_THREADS - 1) bits += eob;  // marker bits appended after the scan
  {
    const int lane = t & 63, wave = t >> 6;
    uint32_t x = bits;
    for (int off = 1; off < 64; off <<= 1) {
      uint32_t y = __shfl_up(x, off, 64);
      if (lane >= off) x += y;
    }
    if (lane == 63) s->wsum[wave] = x;
    __syncthreads();
    uint32_t before = 0;
    for (int w = 0; w < wave; ++w) before += s->wsum[w];
    const uint32_t incl = x + before;
    s->start[t] = incl - bits;
    if (t == ENC_THREADS - 1) s->start[ENC_THREADS] = incl;
  }
  __syncthreads();
  // bit positions from here on count from the aligned word holding the
  // block's first byte: B0 bits of it belong to the previous block
  const uint32_t B0 = 8u * (uint32_t)((uintptr_t)dst & 3);
  const uint32_t total_end = s->start[ENC_THREADS];
  // marker: 3-bit stored header (BFINAL on the stream's last block), pad, 00 00 FF FF
  const uint32_t after = total_end + 3;
  const uint32_t padded = (after + 7) & ~7u;
  const uint32_t block_end = padded + 32;
  if (t == 0 && (block_end >> 3) != plan_bytes) atomicOr(P.fault, 1u);
  BlockWords bw;
  bw.dst = dst - (B0 >> 3);
  bw.lo = B0 >> 3;
  bw.hi = (B0 + block_end) >> 3;
  bw.wlast = (B0 + block_end - 1) >> 5;
  bw.obuf = s->obuf;
  if (ZT_ENC_LDS && bw.wlast >= ENC_OBUF_WORDS) {  // (cannot happen: see ENC_OBUF_WORDS)
    if (t == 0) atomicOr(P.fault, 1u);
    return;
  }
  BitOut bo;
  // thread 0 starts at the header: its complete words come from the slot
  // (block_kernel), then its partial last word
  bo.init(B0 + (t == 0 ? 0u : s->start[t]), bw);
  if (t == 0) {
    bo.first_partial = false;  // word 0's other bytes are the previous block's: stored masked (BlockWords)
    const uint32_t *hw = reinterpret_cast<const uint32_t *>(slot_bytes);
    for (uint32_t k = 0; k < (hdr_bits >> 5); ++k) bo.put(hw[k], 32);
    if (hdr_bits & 31) bo.put(plan->hdr_tail, hdr_bits & 31);
  }
#if ZT_ENC_CACHE
#pragma unroll
  for (int j = 0; j < ENC_CACHE; ++j)
    if ((uint32_t)j < nc) put_token(bo, s, cache[j]);
  for_tokens(tok, a + nc, b, [&](uint32_t tk) { put_token(bo, s, tk); });
#else
  if constexpr (DF_GROUP == 1)
    for_tokens(tok, a, b, [&](uint32_t tk) { put_token(bo, s, tk); });
  else
    for_group_tokens(P, plan, blk, a, b, [&](uint32_t tk) { put_token(bo, s, tk); });
#endif
  if (t == ENC_THREADS - 1) {
    const uint32_t c = s->lit_code[256];
    bo.put(c & 0xFFFF, c >> 16);
    bo.put(last ? 1 : 0, 3);
    bo.put(0, padded - after);
    bo.put(0xFFFF0000u, 32);
  }
  // share the partial first word; the first thread touching a word writes it
  s->first_val[t] = bo.first_partial ? (bo.wrote_first ? bo.first_val : (uint32_t)bo.acc) : 0;
  __syncthreads();
  const bool have_tail = bo.nacc > 0 && !(bo.word == bo.first && bo.first_partial);
  if (have_tail) {
    // this thread started at or before the tail word's first bit: it owns it
    const uint32_t w = bo.word;
    uint32_t v = (uint32_t)bo.acc;
    for (uint32_t u = t + 1; u < ENC_THREADS; ++u) {
      const uint32_t us = B0 + s->start[u], ue = B0 + ((u == ENC_THREADS - 1) ? block_end : s->start[u + 1]);
      if (ue == us) continue;
      if ((us >> 5) != w) break;
      v |= s->first_val[u];
      if (ue >= (w + 1) * 32) break;
    }
    bw.store(w, v);
  }
  if (ZT_ENC_LDS) {
    __syncthreads();
    bw.flush(t);
  }
}

// ================================ 4. stitching ================================
// A restart point (segment boundary) is announced by two empty stored blocks
// after the preceding block (which always ends byte-aligned):
//   00 00 00 FF FF 00 00 00 FF FF
// An ordinary block boundary carries at most one, so the 10-byte pattern at a
// stored-block end marks a segment that inflate may decode on its own.
// (a non-final call -- a shard -- also ends with the marker: the next shard
// is independent when deflated with halo 0, see zt_shard.py)
__device__ __forceinline__ bool restart_after(uint32_t b, uint32_t n, uint32_t restart, int final_,
                                              const uint64_t *span) {
  if (span) {  // batch: inside a stream only (its last block carries BFINAL)
    const uint64_t nx = (uint64_t)(b + 1) * DF_BLOCK;
    return nx < span[2 * (uint64_t)b + 1] && ((nx - span[2 * (uint64_t)b]) / DF_BLOCK) % restart == 0;
  }
  return (b + 1 < n) ? ((b + 1) % restart) == 0 : !final_;
}

__global__ __launch_bounds__(1024) void scan_sizes(const uint32_t *__restrict__ len, uint32_t n,
                                                   uint64_t *__restrict__ off, uint64_t base, uint32_t restart,
                                                   int final_, const uint64_t *__restrict__ span) {
  __shared__ uint64_t part[1024];
  const uint32_t t = threadIdx.x;
  const uint32_t per = (n + 1023) / 1024;
  const uint32_t a = t * per, b = (a + per) < n ? (a + per) : n;
  uint64_t sum = 0;
  for (uint32_t i = a; i < b; ++i) sum += len[i] + (restart_after(i, n, restart, final_, span) ? kRestartMarkerLen : 0);
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
    run += len[i] + (restart_after(i, n, restart, final_, span) ? kRestartMarkerLen : 0);
  }
  if (t == 1023) off[n] = base + part[1023];
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
  int max_chain, nice, lazy, too_far, skip, klen, probe, good, opt;
  int adapt_depth = 0, adapt_thr = 0, adapt_depth2 = 0, adapt_thr2 = 0;  // per-block depth (DeflateParams)
};

static DeflateLevel level_params_base(int level);
static DeflateLevel level_params(int level) {
  DeflateLevel L = level_params_base(level);
  // level 6: per-block depth 6 when at most 40 of the probe's 4096 positions
  // improved at hop 6 or later, else 10 when at most 320 improved at hop 10
  // or later (the 16-window gate: worst window 1.0190 -> 1.0193, source 0.9875
  // -> 0.9904; match per GiB: source text 54.2 -> 44.2 ms, structured 16.6 ->
  // 15.1, the bench corpus 21.0 -> 20.5, wordsalad unchanged;
  // gpurun_out/r06h, tools/adapt_sweep.py)
  if (!getenv("ZT_DF_PARAMS") && (level < 1 || level > 9 || level == 6)) {  // (the levels level_params_base maps to 6)
    L.adapt_depth = 6;
    L.adapt_thr = 40;
    L.adapt_depth2 = 10;
    L.adapt_thr2 = 320;
  }
  // tuning hook: ZT_DF_ADAPT="depth,thr[,depth2,thr2]" (per-block depth; depth 0: off)
  if (const char *e = getenv("ZT_DF_ADAPT")) {
    int d = 0, t = 0, d2 = 0, t2 = 0;
    if (sscanf(e, "%d,%d,%d,%d", &d, &t, &d2, &t2) >= 2) {
      L.adapt_depth = d > 0 && d < L.max_chain ? d : 0;
      L.adapt_thr = t;
      L.adapt_depth2 = L.adapt_depth && d2 > d && d2 < L.max_chain ? d2 : 0;
      L.adapt_thr2 = t2;
    }
  }
  return L;
}
static DeflateLevel level_params_base(int level) {
  // tuning hook: ZT_DF_PARAMS="max_chain,nice,lazy,skip,klen,probe[,good[,opt]]" overrides the level
  if (const char *e = getenv("ZT_DF_PARAMS")) {
    DeflateLevel L{64, 128, 1, 4096, 128, 8, 16, 8, 0};
    if (sscanf(e, "%d,%d,%d,%d,%d,%d,%d,%d", &L.max_chain, &L.nice, &L.lazy, &L.skip, &L.klen, &L.probe, &L.good,
               &L.opt) >= 6)
      return L;
  }
  switch (level) {
    // {max_chain, nice, lazy, too_far, skip, klen, probe, good}: chains on
    // 8-byte keys find the long matches (a 3-byte key chain of the same depth
    // sees mostly candidates that cannot win); near probes (registers) find
    // the short ones; a carried match of `good` bytes cuts the chain to 1/4
    case 1: return {4, 16, 0, 4096, 16, 8, 8, 4, 0};
    case 2: return {8, 32, 0, 4096, 32, 8, 8, 4, 0};
    case 3: return {16, 64, 0, 4096, 64, 8, 16, 4, 0};
    case 4: return {16, 128, 1, 4096, 128, 8, 16, 8, 1};
    case 5: return {24, 128, 1, 4096, 128, 8, 16, 16, 1};
    case 7: return {64, 258, 1, 4096, 258, 8, 16, 16, 1};
    case 8: return {128, 258, 1, 4096, 258, 8, 16, 32, 1};
    case 9: return {512, 258, 1, 4096, 258, 8, 16, 258, 1};
    // 6: chain 28 since matches run past 4 KiB sub-chunk ends (DF_HEAD): the
    // 16-window gate's wordsalad worst 1.0179 (chain 32 without heads:
    // 1.0171), 5 % less chain walking (profiles/r04j_gate.log); 20 since the
    // DP tries cut lengths up to 24 (OP_SHORT): worst window 1.0190, match
    // 24.9 -> 22.4 ms per GiB (chain 18: 1.0225; profiles/r04os_sweep.txt)
    default: return {20, 128, 1, 4096, 128, 8, 16, 16, 1};  // 6
  }
}

// Work split: enough workgroups to cover every CU twice, at most 4 blocks
// (128 KiB) per workgroup (small super-chunks balance uneven data across
// CUs; each loads 28 KiB of history; 1 GiB mixed corpus, match kernel:
// 8 / 4 / 2 blocks 31.8 / 30.7 / 31.4 ms in round 2; round 4: 26.65 / 25.44 /
// 25.75 ms, 16 blocks 29.6, tools/gpu_r04sup.sh), a power of two so segments (32
// blocks) align.
struct DeflateGeom {
  uint32_t nblocks, k, nwg, big_wgs, tail_k;
  size_t res_bytes, slot_bytes, len_bytes, off_bytes, plan_bytes, store_bytes;
};

static size_t deflate_geometry(const DeviceCtx *c, size_t n, DeflateGeom *g) {
  g->nblocks = (uint32_t)((n + DF_BLOCK - 1) / DF_BLOCK);
  if (g->nblocks == 0) g->nblocks = 1;
  uint32_t kk = (g->nblocks + 2 * c->num_cu - 1) / (2 * c->num_cu);
  // tuning hook: ZT_DF_SUPER caps the blocks per workgroup (power of two <= 32)
  static const int cap_env = getenv("ZT_DF_SUPER") ? atoi(getenv("ZT_DF_SUPER")) : 0;
  const uint32_t cap = cap_env > 0 && cap_env <= 32 ? (uint32_t)cap_env : (uint32_t)((128u << 10) / DF_BLOCK);
  uint32_t k2 = 1;
  while (k2 < kk && k2 < cap) k2 <<= 1;
  g->k = k2;
  g->nwg = (g->nblocks + k2 - 1) / k2;
  // the last round of workgroups is the tail where CUs run dry: its blocks go
  // to one-block workgroups (streams identical; 1 GiB bench, match kernel
  // 25.47 -> 24.85 ms; 2-block tail 25.03, two tail rounds 24.92, 8-block
  // workgroups + tail 25.5: tools/gpu_r04tail*.sh).  Tuning hooks:
  // ZT_DF_TAILK = blocks per tail workgroup (0 = none), ZT_DF_TAILR = tail
  // rounds of num_cu workgroups
  static const int tk_env = getenv("ZT_DF_TAILK") ? atoi(getenv("ZT_DF_TAILK")) : -1;
  static const int tr_env = getenv("ZT_DF_TAILR") ? atoi(getenv("ZT_DF_TAILR")) : 1;
  const uint32_t tk = tk_env >= 0 ? (uint32_t)tk_env : 1u;
  g->big_wgs = g->nwg;
  g->tail_k = k2;
  if (tk > 0 && tk < k2 && (k2 % tk) == 0 && tr_env > 0) {
    const uint64_t tail = (uint64_t)tr_env * c->num_cu * k2;
    if ((uint64_t)g->nblocks > tail) {
      g->big_wgs = (uint32_t)((g->nblocks - tail) / k2);
      g->tail_k = tk;
      g->nwg = g->big_wgs + (g->nblocks - g->big_wgs * k2 + tk - 1) / tk;
    }
  }
  g->res_bytes = ((size_t)g->nblocks * DF_BLOCK * 4 + 255) & ~size_t(255);
  g->slot_bytes = (size_t)g->nblocks * DF_SLOT;
  g->len_bytes = ((size_t)g->nblocks * 4 + 255) & ~size_t(255);
  g->off_bytes = ((size_t)(g->nblocks + 1) * 8 + 255) & ~size_t(255);
  g->plan_bytes = ((size_t)g->nblocks * sizeof(BlockPlan) + 255) & ~size_t(255);
  g->store_bytes = ((size_t)g->nblocks + 256 + 255) & ~size_t(255);  // flags + the counter
  return g->res_bytes + g->slot_bytes + g->len_bytes + g->off_bytes + g->plan_bytes + g->store_bytes + 256;
}

// tuning hook: ZT_DF_RESTART = blocks per independent segment (>= 8, rounded
// up to a multiple of the blocks per workgroup)
static uint32_t restart_blocks() {
  static const int e = getenv("ZT_DF_RESTART") ? atoi(getenv("ZT_DF_RESTART")) : 0;
  return e >= 4 ? (uint32_t)e : kRestartBlocks;
}

// classify_kernel runs for the best-of-three block choice (compressionType
// DYNAMIC) with one parse block per DEFLATE block; ZT_DF_CLASSIFY=0 turns it
// off (A/B measurement only)
static bool classify_on(int ctype) {
  static const bool off = getenv("ZT_DF_CLASSIFY") && atoi(getenv("ZT_DF_CLASSIFY")) == 0;
  return ctype == 2 && DF_GROUP == 1 && !off;
}

// bytes per independent segment: a deflate call on a slice that starts at a
// multiple of it (halo 0) writes that slice's part of the whole-buffer stream
size_t deflate_segment_bytes() { return (size_t)restart_blocks() * DF_BLOCK; }

size_t deflate_bound_bytes(size_t n) {
  size_t nb = (n + DF_BLOCK - 1) / DF_BLOCK;
  return n + nb * 16 + (nb / 4 + 1) * kRestartMarkerLen + 64;
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
  DeflateGeom G;
  const size_t need = deflate_geometry(c, n, &G);
  if (need > scratch_size) return set_error(ZT_E_NOMEM, "deflate scratch too small");
  uint8_t *sb = static_cast<uint8_t *>(scratch_base);
  DeflateParams P;
  P.base = d_in - halo;
  P.halo = halo;
  P.end = halo + n;
  P.blocks_per_wg = G.k;
  P.big_wgs = G.big_wgs;
  P.tail_k = G.tail_k;
  P.nblocks = G.nblocks;
  P.restart = (restart_blocks() + G.k - 1) / G.k * G.k;
  // tuning hook: ZT_DF_HIST = KiB of history per super-chunk (multiple of 4, <= 28)
  static const int hist_env = getenv("ZT_DF_HIST") ? atoi(getenv("ZT_DF_HIST")) : 0;
  P.hist_max = hist_env > 0 && hist_env * 1024 <= DF_HIST && hist_env % 4 == 0 ? (uint32_t)hist_env * 1024u
                                                                                : (uint32_t)DF_HIST;
  P.final_ = final_;
  const DeflateLevel L = level_params(level);
  P.max_chain = L.max_chain;
  P.nice_len = L.nice;
  P.lazy = L.lazy;
  P.too_far = L.too_far;
  P.skip_len = L.skip;
  P.klen = L.klen;
  P.probe = L.probe;
  P.good = L.good;
  P.adapt_depth = L.adapt_depth;
  P.adapt_thr = L.adapt_thr;
  P.adapt_depth2 = L.adapt_depth2;
  P.adapt_thr2 = L.adapt_thr2;
  P.ctype = ctype;
  P.opt = L.opt && ctype == 2;
  P.span = nullptr;
  P.res = reinterpret_cast<uint32_t *>(sb);
  P.slots = sb + G.res_bytes;
  P.slot_len = reinterpret_cast<uint32_t *>(sb + G.res_bytes + G.slot_bytes);
  uint64_t *off = reinterpret_cast<uint64_t *>(sb + G.res_bytes + G.slot_bytes + G.len_bytes);
  P.plans = reinterpret_cast<BlockPlan *>(sb + G.res_bytes + G.slot_bytes + G.len_bytes + G.off_bytes);
  P.store = classify_on(ctype) ? sb + G.res_bytes + G.slot_bytes + G.len_bytes + G.off_bytes + G.plan_bytes : nullptr;
  ZT_TRY(timing_begin(c, s, 1));
  P.nstore = reinterpret_cast<uint32_t *>(sb + G.res_bytes + G.slot_bytes + G.len_bytes + G.off_bytes +
                                         G.plan_bytes + ((G.nblocks + 255) & ~255u));
  P.fault = P.nstore + 1;
  ZT_HIP(hipMemsetAsync(P.nstore, 0, 8, s));
  if (P.store) {
    classify_kernel<<<G.nblocks, 256, 0, s>>>(P);
    ZT_HIP(hipGetLastError());
  }
  ZT_TRY(timing_begin(c, s, 0));
  match_kernel<<<G.nwg, DF_THREADS, 0, s>>>(P);
  ZT_HIP(hipGetLastError());
  ZT_TRY(timing_end(c, s, 0));
  if (P.opt) {
    price_kernel<<<G.nblocks, 64, 0, s>>>(P);
    ZT_HIP(hipGetLastError());
    optparse_kernel<<<G.nblocks, 64, 0, s>>>(P);
    ZT_HIP(hipGetLastError());
  }
  parse_kernel<<<G.nblocks, 64, 0, s>>>(P);
  ZT_HIP(hipGetLastError());
  block_kernel<<<G.nblocks, 64, 0, s>>>(P);
  ZT_HIP(hipGetLastError());
  scan_sizes<<<1, 1024, 0, s>>>(P.slot_len, G.nblocks, off, 0, P.restart, final_, nullptr);
  ZT_HIP(hipGetLastError());
  P.out = d_out;
  P.boff = off;
  encode_kernel<<<G.nblocks, ENC_THREADS, 0, s>>>(P);
  ZT_HIP(hipGetLastError());
  ZT_TRY(timing_end(c, s, 1));
  uint64_t total = 0;
  uint32_t nst[2] = {0, 0};  // blocks stored unsearched, encode faults
  {
    void *mb;
    ZT_TRY(mailbox(c, 16, &mb));
    ZT_TRY(x_copy(mb, off + G.nblocks, sizeof total, s));
    ZT_TRY(x_copy((uint8_t *)mb + 8, P.nstore, 8, s));
    ZT_HIP(hipStreamSynchronize(s));
    memcpy(&total, mb, 8);
    memcpy(nst, (uint8_t *)mb + 8, 8);
  }
  if (nst[1]) return set_error(ZT_E_INTERNAL, "deflate: a block's encoded size differs from its plan");
  c->times.blocks_unsearched += nst[0];
  ZT_TRY(timing_collect(c, &c->times.deflate_ms, &c->times.deflate_launches, 0));
  ZT_TRY(timing_collect(c, &c->times.deflate_pipeline_ms, &c->times.deflate_pipelines, 1));
  *out_len = total;
  return ZT_OK;
}

// Batch of independent streams in one pipeline (configs C4 / C2's producer):
// stream f's bytes are at d_in + off[f] (off 32 KiB aligned, increasing, each
// stream's blocks directly after the previous stream's), len[f] > 0.  Every
// workgroup of the match kernel takes one block, so a stream's history never
// reaches into another; each stream's last block carries BFINAL and restart
// markers stay inside streams.  Stream f's bytes land at d_out +
// out_off[f] .. out_off[f + 1] (host array of count + 1).
size_t deflate_batch_scratch_bytes(const DeviceCtx *c, size_t padded) {
  DeflateGeom G;
  const size_t base = deflate_geometry(c, padded, &G);
  return base + (((size_t)G.nblocks * 16 + 255) & ~size_t(255));
}

int deflate_batch_dev_run(DeviceCtx *c, const uint8_t *d_in, size_t count, const uint64_t *off, const uint64_t *len,
                          int ctype, int level, uint8_t *d_out, uint64_t *out_off, void *scratch_base,
                          size_t scratch_size, hipStream_t s) {
  if (count == 0) return ZT_OK;
  const uint64_t padded = off[count - 1] + ((len[count - 1] + DF_BLOCK - 1) / DF_BLOCK) * DF_BLOCK;
  DeflateGeom G;
  const size_t need = deflate_geometry(c, padded, &G);
  const size_t span_bytes = ((size_t)G.nblocks * 16 + 255) & ~size_t(255);
  if (need + span_bytes > scratch_size) return set_error(ZT_E_NOMEM, "deflate scratch too small");
  uint8_t *sb = static_cast<uint8_t *>(scratch_base);
  std::vector<uint64_t> span((size_t)G.nblocks * 2, 0);
  std::vector<uint32_t> first(count);
  for (size_t f = 0; f < count; ++f) {
    const uint64_t b0 = off[f] / DF_BLOCK, nb = (len[f] + DF_BLOCK - 1) / DF_BLOCK;
    if (off[f] % DF_BLOCK || len[f] == 0 || (f && b0 * DF_BLOCK != off[f - 1] + ((len[f - 1] + DF_BLOCK - 1) / DF_BLOCK) * DF_BLOCK))
      return set_error(ZT_E_ARG, "batch streams must be non-empty and packed at 32 KiB boundaries");
    first[f] = (uint32_t)b0;
    for (uint64_t b = b0; b < b0 + nb; ++b) {
      span[2 * b] = off[f];
      span[2 * b + 1] = off[f] + len[f];
    }
  }
  uint64_t *d_span = reinterpret_cast<uint64_t *>(sb + need);
  ZT_HIP(hipMemcpyAsync(d_span, span.data(), span.size() * 8, hipMemcpyHostToDevice, s));
  DeflateParams P;
  P.base = d_in;
  P.halo = 0;
  P.end = padded;
  P.blocks_per_wg = 1;
  P.big_wgs = G.nblocks;
  P.tail_k = 1;
  P.nblocks = G.nblocks;
  P.restart = restart_blocks();
  P.hist_max = DF_HIST;
  P.final_ = 1;
  const DeflateLevel L = level_params(level);
  P.max_chain = L.max_chain;
  P.nice_len = L.nice;
  P.lazy = L.lazy;
  P.too_far = L.too_far;
  P.skip_len = L.skip;
  P.klen = L.klen;
  P.probe = L.probe;
  P.good = L.good;
  P.adapt_depth = L.adapt_depth;
  P.adapt_thr = L.adapt_thr;
  P.adapt_depth2 = L.adapt_depth2;
  P.adapt_thr2 = L.adapt_thr2;
  P.ctype = ctype;
  P.opt = L.opt && ctype == 2;
  P.span = d_span;
  P.res = reinterpret_cast<uint32_t *>(sb);
  P.slots = sb + G.res_bytes;
  P.slot_len = reinterpret_cast<uint32_t *>(sb + G.res_bytes + G.slot_bytes);
  uint64_t *d_off = reinterpret_cast<uint64_t *>(sb + G.res_bytes + G.slot_bytes + G.len_bytes);
  P.plans = reinterpret_cast<BlockPlan *>(sb + G.res_bytes + G.slot_bytes + G.len_bytes + G.off_bytes);
  P.store = classify_on(ctype) ? sb + G.res_bytes + G.slot_bytes + G.len_bytes + G.off_bytes + G.plan_bytes : nullptr;
  ZT_TRY(timing_begin(c, s, 1));
  P.nstore = reinterpret_cast<uint32_t *>(sb + G.res_bytes + G.slot_bytes + G.len_bytes + G.off_bytes +
                                         G.plan_bytes + ((G.nblocks + 255) & ~255u));
  P.fault = P.nstore + 1;
  ZT_HIP(hipMemsetAsync(P.nstore, 0, 8, s));
  if (P.store) {
    classify_kernel<<<G.nblocks, 256, 0, s>>>(P);
    ZT_HIP(hipGetLastError());
  }
  ZT_TRY(timing_begin(c, s, 0));
  match_kernel<<<G.nblocks, DF_THREADS, 0, s>>>(P);
  ZT_HIP(hipGetLastError());
  ZT_TRY(timing_end(c, s, 0));
  if (P.opt) {
    price_kernel<<<G.nblocks, 64, 0, s>>>(P);
    ZT_HIP(hipGetLastError());
    optparse_kernel<<<G.nblocks, 64, 0, s>>>(P);
    ZT_HIP(hipGetLastError());
  }
  parse_kernel<<<G.nblocks, 64, 0, s>>>(P);
  ZT_HIP(hipGetLastError());
  block_kernel<<<G.nblocks, 64, 0, s>>>(P);
  ZT_HIP(hipGetLastError());
  scan_sizes<<<1, 1024, 0, s>>>(P.slot_len, G.nblocks, d_off, 0, P.restart, 1, d_span);
  ZT_HIP(hipGetLastError());
  P.out = d_out;
  P.boff = d_off;
  encode_kernel<<<G.nblocks, ENC_THREADS, 0, s>>>(P);
  ZT_HIP(hipGetLastError());
  ZT_TRY(timing_end(c, s, 1));
  std::vector<uint64_t> boff((size_t)G.nblocks + 1);
  uint32_t nst[2] = {0, 0};  // blocks stored unsearched, encode faults
  {
    void *mb;
    const size_t bb = boff.size() * 8;
    ZT_TRY(mailbox(c, bb + 8, &mb));
    ZT_TRY(x_copy(mb, d_off, bb, s));
    ZT_TRY(x_copy((uint8_t *)mb + bb, P.nstore, 8, s));
    ZT_HIP(hipStreamSynchronize(s));
    memcpy(boff.data(), mb, bb);
    memcpy(nst, (uint8_t *)mb + bb, 8);
  }
  if (nst[1]) return set_error(ZT_E_INTERNAL, "deflate: a block's encoded size differs from its plan");
  c->times.blocks_unsearched += nst[0];
  ZT_TRY(timing_collect(c, &c->times.deflate_ms, &c->times.deflate_launches, 0));
  ZT_TRY(timing_collect(c, &c->times.deflate_pipeline_ms, &c->times.deflate_pipelines, 1));
  for (size_t f = 0; f < count; ++f) out_off[f] = boff[first[f]];
  out_off[count] = boff[G.nblocks];
  return ZT_OK;
}

#ifdef ZT_DF_TIME
extern "C" int zt_debug_df_time(unsigned long long *out) {
  (void)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_df_time), sizeof(unsigned long long) * 8);
  unsigned long long z[8] = {};
  (void)hipMemcpyToSymbol(HIP_SYMBOL(g_df_time), z, sizeof z);
  return 0;
}
#endif

#ifdef ZT_DF_TIME
extern "C" int zt_debug_bk_time(unsigned long long *out) {
  (void)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_bk_time), sizeof(unsigned long long) * 8);
  unsigned long long z[8] = {};
  (void)hipMemcpyToSymbol(HIP_SYMBOL(g_bk_time), z, sizeof z);
  return 0;
}
#endif

#ifdef ZT_DF_COUNT
extern "C" int zt_debug_df_count(unsigned long long *out) {
  (void)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_df_count), sizeof(unsigned long long) * 8);
  unsigned long long z[8] = {};
  (void)hipMemcpyToSymbol(HIP_SYMBOL(g_df_count), z, sizeof z);
  return 0;
}
#endif

size_t deflate_scratch_bytes(const DeviceCtx *c, size_t n) {
  DeflateGeom G;
  return deflate_geometry(c, n, &G);
}

}  // namespace zt
