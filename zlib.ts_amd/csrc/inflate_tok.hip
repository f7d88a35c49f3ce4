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
#include "inflate_simt.h"

namespace zt {

namespace {


struct TokShared {
  uint32_t inbuf[IN_RING_WORDS + 4];
  HuffTab lit;
  HuffTab dist;
  uint8_t lens[320];
#ifdef ZT_TOK_LDS_PAD
  uint8_t pad[ZT_TOK_LDS_PAD];  // (measurement: occupancy held to a larger table's)
#endif
};


// 3 waves per SIMD: the register budget (<= 168 VGPRs) the body decoder
// fits in; the compiler's own choice drifts to 169+ (2 waves) on small edits
#ifndef ZT_TOK_WAVES
#define ZT_TOK_WAVES 3
#endif
#define ZT_TOK_ATTR __attribute__((amdgpu_waves_per_eu(ZT_TOK_WAVES)))
__global__ __launch_bounds__(64) ZT_TOK_ATTR void tokenize_kernel(TokParams P) {
  __shared__ TokShared sh;
  __shared__ SpecShared spsh;
  const uint32_t u = P.order ? P.order[blockIdx.x] : blockIdx.x;
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
  bool any_run = false;  // run tokens written (flag bit 31 of the result's ntok: expand_kernel's run path)
  bool other = false;    // tokens that are not runs (bit 30 of ntok: every output byte comes from a run)
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
        if (P.run_tokens && len >= kStoredRunMin) {
          // a long payload stays in the input: three run tokens, and
          // expand_kernel writes its literal descriptors from there
          to.emit(len << 16);
          to.emit((uint32_t)p);
          to.emit((uint32_t)(p >> 32));
          any_run = true;
        } else {
          other = true;
          to.flush_partial();
          for (uint32_t j = lane; j < len; j += 64) to.tok[nt0 + j] = gin[p + j];
          const uint32_t nt = nt0 + len;
          const uint32_t idx = (nt & ~63u) + (uint32_t)lane;
          if ((uint32_t)lane < (nt & 63) && idx >= nt0) to.stg = gin[p + idx - nt0];
          to.ntok = nt;
        }
        op += len;
      }
      rd.seek_byte(p + len);
    } else {
      other = true;
      status = read_tables<false>(rd, sh.lens, &sh.lit, &sh.dist, btype, lane, detail);
      if (status) break;
      uint64_t end_bit = 0;
      const uint64_t body0 = rd.pos_bits();
      const uint32_t nt_before = uni(to.ntok);
      const uint64_t op_before = op;
      uint32_t *dump = (P.dbg && u == P.dump_unit && P.dump_once == 0) ? reinterpret_cast<uint32_t *>(P.dbg + (uint64_t)P.count * 8) : nullptr;
      int r = P.simt ? tok_huffman_simt<true>(rd, body0, &sh.lit, &sh.dist, to, op, &spsh, end_bit, dump) : 1;
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
    r.ntok = to.ntok | (any_run ? 0x80000000u : 0u) | (any_run && !other ? 0x40000000u : 0u);
    r.status = status;
    r.detail = detail;
    r.stop_idx = stop_idx;
    P.res[u] = r;
  }
}

// ---------------------------------------------------------------- phase B

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

// A descriptor copied from an earlier byte of the same copy step is used by a
// later byte.  A ring read more than 32768 - CP_STEP back could then hit a slot
// this step has already overwritten (a match chain reaching up to 32 KiB +
// 255 back), so such a copy becomes an in-step reference to the byte it came
// from, which copy_kernel resolves from the step itself.
__device__ __forceinline__ uint32_t safe_desc(uint32_t d, uint32_t step_off) {
  return ((d & 0x8000u) || d < 32768u - CP_STEP) ? d : (0xC000u | step_off);
}

struct ExpandShared {
  uint32_t tok[RS_TOK_RING];   // token chunks, filled by LDS-DMA
  uint32_t mark[64];
  uint16_t cw[CP_STEP];        // descriptors of the current copy step
};

// RUNS: the unit holds run tokens (ChainUnit ntok bit 31); units without
// them take the loop without the run checks
template <bool RUNS>
__device__ __forceinline__ void expand_unit(const ResolveParams &P, ExpandShared &sh, const ChainUnit &cu) {
  const uint32_t u = P.order ? P.order[blockIdx.x] : blockIdx.x;
  const int lane = threadIdx.x & 63;
  const uint32_t *tk = P.tokens + cu.tok_off;
  const uint32_t ntok = cu.ntok & 0x3FFFFFFFu;
  const uint32_t nchunks = (ntok + 63) / 64;
  uint16_t *desc = P.desc + cu.desc_off;
  const uint64_t back = cu.out_off - cu.seg_off;  // bytes of the segment before this unit
  const bool behind_ok = P.marker && cu.seg_off != 0;  // general path: not the stream's first segment
  sh.mark[lane] = 0;
  uint32_t seq = 0;
  uint32_t issued = 0;
  uint32_t op = 0;  // unit-relative output position
  bool bad = false;
  // The scan of 64 token lengths is kept across windows: a window takes its
  // bytes from the scan while the scan covers the whole window (a 64-token
  // scan spans several windows but for literal-only stretches), and the
  // tokens are re-read and re-scanned from the one holding the next byte
  // only when it does not.  Scan coordinates: byte 0 = token cb's first byte.
  uint32_t cb = 0;      // the scan's first token
  uint32_t B = 0;       // scan coordinate of the next output byte
  uint32_t j0 = 0;      // the scan's tokens that end at or before B
  uint32_t T = 0;       // bytes the scan covers (up to its first stored run)
  bool last = false;    // the scan holds the unit's last token (and no run)
  bool scanned = false;
  uint32_t t = 0, len = 0, S = 0;
  bool valid = false;
  while (cb + j0 < ntok) {
    const uint64_t pos = back + op;  // segment position of this window's first byte
    // windows coincide with copy_kernel's 64-byte steps of the segment
    const uint32_t room = 64 - (uint32_t)(pos & 63);
    if (!scanned || (T - B < room && !last)) {
      // (re)scan from the token holding byte B; rem of its bytes are done
      const uint32_t cur = cb + j0;
      const uint32_t rem = j0 < 64 && scanned ? B - (uint32_t)__builtin_amdgcn_readlane((int)(S - len), j0) : 0u;
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
      valid = ti < ntok;
      t = sh.tok[ti & (RS_TOK_RING - 1)];
      // a stored run at the cursor (tokenize_kernel: len << 16 with distance 0,
      // then the payload's input offset in two tokens): its literal descriptors
      // straight from the input, 8 bytes per lane in flight
      const uint32_t t0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)t);
      if (RUNS && rem == 0 && (t0 >> 16) != 0 && (t0 & 0xFFFFu) == 0) {
        const uint32_t rl = t0 >> 16;
        const uint64_t src = (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)t, 1) |
                             ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)t, 2) << 32);
        const uint8_t *sp = P.in + src;
        for (uint32_t i0 = 0; i0 < rl; i0 += 512) {
          uint32_t b[8];
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            const uint32_t i = i0 + 64 * k + (uint32_t)lane;
            b[k] = i < rl ? sp[i] : 0u;
          }
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            const uint32_t i = i0 + 64 * k + (uint32_t)lane;
            if (i < rl) desc[op + i] = (uint16_t)(0x8000u | b[k]);
          }
        }
        // the copy step holding the run's end keeps its descriptors for the
        // references of the tokens after it
        const uint64_t e = pos + rl;
        const uint64_t ws_e = (e - 1) & ~uint64_t(CP_STEP - 1);
        for (uint64_t x = (pos > ws_e ? pos : ws_e) + (uint64_t)lane; x < e; x += 64)
          sh.cw[x - ws_e] = (uint16_t)(0x8000u | sp[x - pos]);
        wave_sync();
        op += rl;
        cb = cur + 3;
        j0 = 0;
        B = 0;
        scanned = false;
        continue;
      }
      len = valid ? tok_len(t) : 0u;
      S = wave_incl_scan(len);
      T = (uint32_t)__builtin_amdgcn_readlane((int)S, 63);
      last = cur + 64 >= ntok;
      // the scan ends where a stored run starts (the run is taken at the
      // cursor); the run's two offset tokens after it are never scanned into one
      const uint64_t runs = RUNS ? __ballot(valid && (t >> 16) != 0 && (t & 0xFFFFu) == 0) : 0ull;
      if (RUNS && runs) {
        const int fl = __ffsll((long long)runs) - 1;  // >= 1: a run at the cursor was taken above
        T = (uint32_t)__builtin_amdgcn_readlane((int)(S - len), fl);
        last = false;
      }
      cb = cur;
      B = rem;
      j0 = 0;
      scanned = true;
    }
    const uint32_t W = T - B < room ? T - B : room;
    const uint64_t ws = pos & ~uint64_t(CP_STEP - 1);
    ++seq;
    // tokens that end inside the window mark the next token's start
    const int32_t p = (int32_t)S - (int32_t)B;
    if (valid && p > 0 && p < 64) sh.mark[p] = seq;
    wave_sync();
    const uint64_t starts = __ballot(sh.mark[lane] == seq);
    const uint32_t owner = j0 + __popcll(starts & (~0ull >> (63 - lane)));  // token of byte `lane`
    const uint32_t tj = bperm(t, owner);
    const uint32_t ej = bperm(S - len, owner);  // the token's start (scan coordinates)
    // descriptor: 0x8000 | byte (literal), 0xC000 | o (= byte ws + o, before
    // this unit), or ws - src - 1 (a byte before the copy step); references
    // into the step are followed here (earlier windows from LDS, this window
    // by pointer jumping over the lanes)
    // Branch-free, in step-relative 32-bit offsets: the window lies inside
    // one copy step (po + lane < CP_STEP) and a source is at most 32768 + 257
    // bytes back.  k / dist in single precision: (k + 0.5) / dist is at
    // least 0.5 / dist from an integer, far above v_rcp_f32's error at
    // k < 258 (the quotient only matters when k >= dist, i.e. dist < 258).
    const uint32_t po = (uint32_t)(pos - ws);
    const uint32_t bo = back > ws ? (uint32_t)(back - ws) : 0u;
    const bool near_start = pos < 65536u && !behind_ok;
    const bool match = (uint32_t)lane < W && (tj >> 16) != 0;
    const uint32_t dist = tj & 0xFFFF;
    const uint32_t k = B + (uint32_t)lane - ej;  // byte index inside the match
    const uint32_t kq = (uint32_t)(((float)k + 0.5f) * __builtin_amdgcn_rcpf((float)dist));  // k / dist
    const uint32_t D = __umul24(dist, kq + 1u);
    const bool b = match && near_start && D > (uint32_t)pos + (uint32_t)lane;  // reaches behind the segment start
    bad = bad || b;
    // (marker segments: a source before the segment start is a byte of the
    // previous segment's last 32 KiB, D <= 32768 keeps it in the ring)
    const int32_t so = (int32_t)(po + (uint32_t)lane) - (int32_t)D;  // source, relative to the step
    const uint32_t cwv = sh.cw[so < 0 ? 0u : (uint32_t)so & (CP_STEP - 1)];  // (an earlier window's)
    const uint32_t dm = so < 0 ? (uint32_t)(-so - 1)                         // before the copy step
                        : so < (int32_t)bo ? (0xC000u | (uint32_t)so)          // before this unit: copy_kernel resolves it
                                           : safe_desc(cwv, (uint32_t)so);
    const bool m_ok = match && !b;
    uint32_t dsc = m_ok ? dm : 0x8000u | (tj & 0xFF);  // (lanes past W: never read or written)
    int32_t ptr = m_ok && so >= (int32_t)po ? so - (int32_t)po : -1;
    const uint32_t first = (uint32_t)so;  // step offset of the byte's direct source
    const bool jumped = ptr >= 0;
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
    if (jumped) dsc = safe_desc(dsc, first);
    if ((uint32_t)lane < W) {
      desc[op + lane] = (uint16_t)dsc;
      sh.cw[po + lane] = (uint16_t)dsc;
    }
    wave_sync();
    op += W;
    B += W;
    j0 = (uint32_t)__popcll(__ballot(valid && S <= B));
  }
  const bool any_bad = __ballot(bad) != 0;
  if (lane == 0) P.unit_status[u] = any_bad ? ZT_E_INVALID_DISTANCE : (op != cu.out_len ? ZT_E_INPUT_BROKEN : ZT_OK);
}

// bytes [src, src + n) to [dst, dst + n) by one wave: dst-aligned words
// (each from two aligned source words), 4 per lane in flight
__device__ __forceinline__ void wave_copy(uint8_t *dst, const uint8_t *src, uint32_t n, int lane) {
  const uint32_t h = ((4u - (uint32_t)((uintptr_t)dst & 3)) & 3) < n ? ((4u - (uint32_t)((uintptr_t)dst & 3)) & 3) : n;
  if ((uint32_t)lane < h) dst[lane] = src[lane];
  const uint32_t n4 = (n - h) / 4;
  const uint8_t *s = src + h;
  uint32_t *d4 = reinterpret_cast<uint32_t *>(dst + h);
  const uint32_t sh = (uint32_t)((uintptr_t)s & 3);
  const uint32_t *s4 = reinterpret_cast<const uint32_t *>(s - sh);
  // source words [0, nw) exist: the last one a full word only when the copy
  // reaches it (no read past the payload's last byte)
  const uint32_t nsrc = (sh + 4 * n4 + 3) / 4;
  for (uint32_t w0 = 0; w0 < n4; w0 += 256) {
    uint32_t v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint32_t w = w0 + 64 * k + (uint32_t)lane;
      uint32_t lo = 0, hi = 0;
      if (w < n4) {
        lo = s4[w];
        hi = sh && w + 1 < nsrc ? s4[w + 1] : 0u;
      }
      v[k] = sh ? __builtin_amdgcn_alignbyte(hi, lo, sh) : lo;
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint32_t w = w0 + 64 * k + (uint32_t)lane;
      if (w < n4) d4[w] = v[k];
    }
  }
  for (uint32_t i = h + 4 * n4 + (uint32_t)lane; i < n; i += 64) dst[i] = src[i];
}

// a unit whose every output byte is a stored run, in a segment of such units
// (ChainUnit ntok bit 30, set by the host): the runs go from the input
// straight to their final place (copy_kernel skips the segment) -- 1 byte
// read and 1 written per byte instead of descriptors written and read back
__device__ __forceinline__ void expand_direct(const ResolveParams &P, const ChainUnit &cu) {
  const int lane = threadIdx.x & 63;
  const uint32_t *tk = P.tokens + cu.tok_off;
  const uint32_t ntok = cu.ntok & 0x3FFFFFFFu;
  uint32_t op = 0;
  bool ok = ntok % 3 == 0;
  for (uint32_t i = 0; ok && i < ntok; i += 3) {
    const uint32_t t0 = tk[i], lo = tk[i + 1], hi = tk[i + 2];
    const uint32_t rl = t0 >> 16;
    if ((t0 & 0xFFFFu) || rl == 0 || op + rl > cu.out_len) {
      ok = false;
      break;
    }
    const uint64_t src = (uint64_t)lo | ((uint64_t)hi << 32);
    wave_copy(P.out + cu.out_off + op, P.in + src, rl, lane);
    op += rl;
  }
  if (lane == 0) P.unit_status[P.order ? P.order[blockIdx.x] : blockIdx.x] = ok && op == cu.out_len ? ZT_OK : ZT_E_INPUT_BROKEN;
}

__global__ __launch_bounds__(64) void expand_kernel(ResolveParams P) {
  __shared__ ExpandShared sh;
  if (P.info && !P.info->ok) return;  // the host walks the chain instead
  const ChainUnit cu = P.units[P.order ? P.order[blockIdx.x] : blockIdx.x];
  if ((cu.ntok >> 30) == 3u)
    expand_direct(P, cu);
  else if (cu.ntok >> 31)
    expand_unit<true>(P, sh, cu);
  else
    expand_unit<false>(P, sh, cu);
}


typedef unsigned int u32x4r __attribute__((ext_vector_type(4)));


struct CopyShared {
  uint8_t ring[RING];                        // 32 KiB history, also the output staging
  uint16_t desc[CP_DESC_RING];               // descriptor chunks, filled by LDS-DMA
};

// ring bytes [lo, hi) (segment positions) to out + lo
template <typename U>
__device__ __forceinline__ void cp_flush(const CopyShared *sh, uint8_t *out, U lo, U hi, int lane) {
  if (lo >= hi) return;
  if (hi - lo == RS_FLUSH && (((uintptr_t)out + lo) & 15) == 0) {
    // a whole granule: every ring read in flight before the stores
    constexpr int K = RS_FLUSH / 1024;
    u32x4r v[K];
    uint8_t *o = out + lo;
#pragma unroll
    for (int k = 0; k < K; ++k)
      v[k] = *reinterpret_cast<const u32x4r *>(&sh->ring[((uint32_t)lo + (uint32_t)lane * 16 + 1024 * k) & RING_MASK]);
#pragma unroll
    for (int k = 0; k < K; ++k) *reinterpret_cast<u32x4r *>(o + (uint32_t)lane * 16 + 1024 * k) = v[k];
  } else if ((((uintptr_t)out + lo) & 15) == 0 && ((hi - lo) & 15) == 0) {
    for (U p = lo + (U)lane * 16; p < hi; p += 1024)
      *reinterpret_cast<u32x4r *>(out + p) = *reinterpret_cast<const u32x4r *>(&sh->ring[p & RING_MASK]);
  } else {
    for (U p = lo + lane; p < hi; p += 64) out[p] = sh->ring[p & RING_MASK];
  }
}

// one descriptor -> byte, or -1 for "the byte op + off of this step"
// (branch-free: the ring is read for every descriptor, the literal selected
// after -- per-byte branches cost more issue slots than the extra LDS read)
__device__ __forceinline__ uint32_t cp_byte(const CopyShared *sh, uint64_t op, uint32_t d, int32_t &off) {
  const uint32_t rv = sh->ring[((uint32_t)op - d - 1) & RING_MASK];
  const bool lit = (d & 0x8000u) != 0;
  off = (lit && (d & 0x4000u)) ? (int32_t)(d & 0x3FF) : -1;  // 0xC000 | o: the byte op + o of this step
  return lit ? (d & 0xFF) : rv;
}

// the two descriptors of a dword (low half first) -> their bytes in bits
// 0-7 of lo / hi (bits 8-31 left unspecified).  A literal is selected by its
// sign-extended bit 15 in one 3-input bit select (v_bitop3) instead of a
// compare and a VCC select; the low half's ring index needs no extract
// ((opm1 - x) mod 2^15 = (opm1 - d0) mod 2^15).  Only for steps with no
// in-step reference.
__device__ __forceinline__ void cp_pair(const CopyShared *sh, uint32_t opm1, uint32_t x, uint32_t &lo, uint32_t &hi) {
  const uint32_t d1 = x >> 16;
  const uint32_t r0 = sh->ring[(opm1 - x) & RING_MASK];
  const uint32_t r1 = sh->ring[(opm1 - d1) & RING_MASK];
  const uint32_t m0 = (uint32_t)__builtin_amdgcn_sbfe((int)x, 15, 1);  // ~0: a literal
  const uint32_t m1 = (uint32_t)((int32_t)x >> 31);
  lo = __builtin_amdgcn_bitop3_b32(m0, x, r0, 0xCA);  // m ? a : b, bitwise
  hi = __builtin_amdgcn_bitop3_b32(m1, d1, r1, 0xCA);
}

#ifdef ZT_CP_TIME
__device__ unsigned long long g_cp_time[8];  // debug: copy_kernel cycles per phase (lane 0 of each wave), [6] steps, [7] waves
#define CP_T(v) v = __builtin_readcyclecounter()
#else
#define CP_T(v) (void)0
#endif
// one segment's bytes [0, n) from its descriptors; U is the offset type
// (uint32_t below 2^31 bytes: the per-step bookkeeping is 32-bit)
template <typename U>
__device__ __forceinline__ void copy_run(CopyShared &sh, uint8_t *out, const uint16_t *dsrc, const U n, const int lane) {
#ifdef ZT_CP_TIME
  unsigned long long cp_acc[4] = {0, 0, 0, 0}, ct0 = 0, ct1 = 0, ct2 = 0, ct3 = 0, ct4 = 0, nsteps = 0;
#endif
  U issued = 0, flushed = 0;
  // lane j: bytes op + 256 g + 4 j .. + 3 for each group g (bytes past n are
  // never flushed).  The next step's descriptors are fetched and read right
  // after this step's ring writes, so a step starts with its ring reads.
  uint64_t dd[CP_G];
  auto read_desc = [&](U o) {
#pragma unroll
    for (int g = 0; g < CP_G; ++g) {
      const uint32_t x = (uint32_t)o + 256u * g + 4 * (uint32_t)lane;  // ring / descriptor index (masked)
      dd[g] = *reinterpret_cast<const uint64_t *>(&sh.desc[x & (CP_DESC_RING - 1)]);
    }
  };
  if (n) {
    cp_desc_fetch<U>(dsrc, sh.desc, 0, n, issued, lane);
    read_desc(0);
  }
  for (U op = 0; op < n; op += CP_STEP) {
    CP_T(ct0);
    // every byte of a step is a literal or a ring byte before the step, so
    // all ring reads are issued before any write
    // (an in-step reference 0xC000 | o is the only descriptor with bits 15
    // and 14 both set: one AND with its own shift per dword finds any)
    uint32_t bw[CP_G];
    uint32_t refs = 0;
    const uint32_t opm1 = (uint32_t)op - 1;
#pragma unroll
    for (int g = 0; g < CP_G; ++g) {
      const uint32_t x0 = (uint32_t)dd[g], x1 = (uint32_t)(dd[g] >> 32);
      refs |= (x0 & (x0 << 1)) | (x1 & (x1 << 1));
      uint32_t b0, b1, b2, b3;
      cp_pair(&sh, opm1, x0, b0, b1);
      cp_pair(&sh, opm1, x1, b2, b3);
      // bytes 0 of b0, b1 and of b2, b3 side by side, the pairs joined
      bw[g] = __builtin_amdgcn_perm(b1, b0, 0x0C0C0400u) | (__builtin_amdgcn_perm(b3, b2, 0x0C0C0400u) << 16);
    }
    const bool in_step = (refs & 0x80008000u) != 0;
    CP_T(ct2);
    if (__ballot(in_step) == 0) {
#pragma unroll
      for (int g = 0; g < CP_G; ++g)
        *reinterpret_cast<uint32_t *>(&sh.ring[((uint32_t)op + 256u * g + 4 * (uint32_t)lane) & RING_MASK]) = bw[g];
    } else {
      // a unit boundary inside this step left references into it: resolve
      // them byte by byte (64-byte sub-steps, pointer jumping)
      for (uint32_t sub = 0; sub < CP_STEP; sub += 64) {
        const U y = op + sub + (U)lane;
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
    CP_T(ct3);
    if (op + CP_STEP < n) {
      cp_desc_fetch<U>(dsrc, sh.desc, op + CP_STEP, n, issued, lane);
      read_desc(op + CP_STEP);
    }
    CP_T(ct1);
    const U end = op + CP_STEP < n ? op + CP_STEP : n;
    if (end - flushed >= RS_FLUSH) {
      const U upto = flushed + RS_FLUSH;
      cp_flush(&sh, out, flushed, upto, lane);
      flushed = upto;
#ifdef ZT_CP_FLUSH_WAIT
      __builtin_amdgcn_s_waitcnt(0x0F70);  // keep vmcnt counting descriptor chunks only
#endif
      // (no wait here: vector memory operations retire in issue order, so the
      // counted descriptor waits above only wait longer with the stores in
      // flight, never shorter)
    }
#ifdef ZT_CP_TIME
    CP_T(ct4);
    cp_acc[0] += ct1 - ct3;
    cp_acc[1] += ct2 - ct0;
    cp_acc[2] += ct3 - ct2;
    cp_acc[3] += ct4 - ct1;
    ++nsteps;
#endif
  }
#ifdef ZT_CP_TIME
  if (lane == 0) {
    for (int k = 0; k < 4; ++k) atomicAdd(&g_cp_time[k], cp_acc[k]);
    atomicAdd(&g_cp_time[6], nsteps);
    atomicAdd(&g_cp_time[7], 1ull);
  }
#endif
  wave_sync();
  cp_flush(&sh, out, flushed, n, lane);
}

__global__ __launch_bounds__(64) void copy_kernel(ResolveParams P) {
  __shared__ CopyShared sh;
  const uint32_t sg = blockIdx.x;
  const int lane = threadIdx.x & 63;
  // device-built chain: launched for the bound on its segments
  if (P.info && (!P.info->ok || sg >= P.info->nseg)) return;
  SegJob sj = P.segs[sg];
  if (sj.count >> 31) {  // stored runs only: expand_kernel wrote the bytes
    if (lane == 0) P.seg_status[sg] = ZT_OK;
    return;
  }
  const uint64_t seg_out = P.units[sj.first].out_off;
  const ChainUnit lastu = P.units[sj.first + sj.count - 1];
  const uint64_t n = lastu.out_off + lastu.out_len - seg_out;  // segment bytes
  uint8_t *out = P.out + seg_out;
  const uint16_t *dsrc = P.desc + P.units[sj.first].desc_off;  // 512-aligned (cp_desc_fetch's chunks)
  if (n < (1ull << 31))
    copy_run<uint32_t>(sh, out, dsrc, (uint32_t)n, lane);
  else
    copy_run<uint64_t>(sh, out, dsrc, n, lane);
  if (lane == 0) P.seg_status[sg] = ZT_OK;
}

}  // namespace

int tokenize_units_dev(const TokParams &p, hipStream_t s) {
  if (p.count == 0) return ZT_OK;
  tokenize_kernel<<<p.count, 64, 0, s>>>(p);
  ZT_HIP(hipGetLastError());
  return ZT_OK;
}

#ifdef ZT_TK_TIME
extern "C" int zt_debug_tk_time(unsigned long long *out) {
  (void)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_tk_time), sizeof(unsigned long long) * 8);
  unsigned long long z[8] = {};
  (void)hipMemcpyToSymbol(HIP_SYMBOL(g_tk_time), z, sizeof z);
  return 0;
}
#endif

#ifdef ZT_CP_TIME
extern "C" int zt_debug_cp_time(unsigned long long *out) {
  (void)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_cp_time), sizeof(unsigned long long) * 8);
  unsigned long long z[8] = {};
  (void)hipMemcpyToSymbol(HIP_SYMBOL(g_cp_time), z, sizeof z);
  return 0;
}
#endif

int expand_units_dev(const ResolveParams &p, hipStream_t s) {
  if (p.nunits == 0) return ZT_OK;
  expand_kernel<<<p.nunits, 64, 0, s>>>(p);
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
