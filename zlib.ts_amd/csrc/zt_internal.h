// zt_internal.h -- shared host/device helpers for libzt (not installed).
#pragma once
#include <functional>
#include <mutex>
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>
#include <string>
#include <vector>

#include "../../include/zt.h"

namespace zt {

// ---- error plumbing -------------------------------------------------------
int set_error(int code, const std::string &msg);
int hip_fail(hipError_t e, const char *what);

#define ZT_HIP(call)                                       \
  do {                                                     \
    hipError_t e_ = (call);                                \
    if (e_ != hipSuccess) return ::zt::hip_fail(e_, #call); \
  } while (0)

#define ZT_TRY(call)      \
  do {                    \
    int rc_ = (call);     \
    if (rc_) return rc_;  \
  } while (0)

// ---- per-device context -----------------------------------------------------
// checksum_segments' in-kernel merge (checksum.hip): zero between calls
// checksum merge (checksum.hip): each workgroup's partial sums in its own
// slot, then group tickets (128 bytes apart) and one top ticket -- the last
// workgroup to arrive reduces the slots
constexpr int kCkGroups = 32;
constexpr int kCkMaxWg = 4096;  // checksums_dev's grid: at most num_cu * 8
struct CkPart {
  unsigned long long s1, s2;
  uint32_t crc, pad[3];
};
struct CkAcc {
  uint32_t grp[kCkGroups * 32];
  uint32_t done, pad[31];
  CkPart part[kCkMaxWg];
};

// One default stream per device plus grow-only scratch buffers, so the
// host-pointer entry points do not hipMalloc on every call.
struct DeviceCtx {
  // host entry points hold it for their whole call: scratch, pinned staging
  // and the streams are shared by every thread that uses this device
  std::recursive_mutex mu;
  int device = -1;  // logical device (zt_set_device index)
  int phys = -1;    // HIP device it runs on (differs only under ZT_ALIAS_DEVICES)
  hipStream_t stream = nullptr;
  int num_cu = 0;
  // checksum constants (uploaded once)
  uint32_t *d_crc_nib = nullptr;    // nibble tables (ZT_CRC_NIB_N entries)
  uint32_t *d_crc_x2n = nullptr;    // x^(2^k) mod P, k = 0..31
  uint32_t *d_crc_shift = nullptr;  // checksum.hip merge constants (crc_shift_tables)
  CkAcc *d_ck_acc = nullptr;        // checksum merge accumulators (zeroed once, left zeroed by every call)
  // scratch
  static constexpr int kSlots = 29;
  void *d_buf[kSlots] = {};  // slot 8: checksum segment partials; 10-17: general inflate (inflate_gen.hip);
                             // 20: segment inflate's sync-point sort (inflate_seg.hip); 21: stored runs;
                             // 22: pipelined host inflate's output, 23-25: its overflow ring (inflate_api.cpp);
                             // 26: general inflate's window pointer-jumping buffers; 27: framed batch members;
                             // 28: segment inflate's tokenize launch order
  size_t buf_size[kSlots] = {};
  // second stream: checksums run beside the deflate pipeline in the containers
  hipStream_t aux = nullptr;
  hipEvent_t aux_ev = nullptr;
  void *h_pinned[10] = {};  // pinned host staging: 0 batch data, 1 inflate metadata, 2-3 upload/download chunks,
                            // 4-5 download chunks of the three-stage pipeline (pipeline_h2d_d2h),
                            // 6-7 second input group / output group of a grouped batch (batch_api.cpp),
                            // 8 the readback mailbox (mailbox())
  hipEvent_t xfer_ev[4] = {};  // chunk buffer 2 + k's copy has finished
  hipStream_t up = nullptr, dn = nullptr;  // pipeline_h2d_d2h: H2D and D2H copy streams
  // zt_timing_enable: HIP-event kernel timing
  bool timing = false;
  hipEvent_t ev[8] = {};  // [2k, 2k+1]: interval k (0 match, 1 deflate pipeline, 2 inflate)
  zt_kernel_times times = {};
  size_t pinned_size[10] = {};
};

// Records the begin / end event of interval k (0 or 1) when timing is on.
int timing_begin(DeviceCtx *c, hipStream_t s, int k = 0);
int timing_end(DeviceCtx *c, hipStream_t s, int k = 0);
// After the stream is synchronized: adds interval k's elapsed time to *acc.
int timing_collect(DeviceCtx *c, double *acc_ms, uint64_t *count, int k = 0);

// Context of the calling thread's current device (created on first use).
int get_ctx(DeviceCtx **out);
// Grow-only device scratch slot `slot` to at least `bytes`.
int scratch(DeviceCtx *c, int slot, size_t bytes, void **ptr);
// Grow-only pinned host staging buffer `slot` (0 or 1) of at least `bytes`.
int pinned(DeviceCtx *c, size_t bytes, void **ptr, int slot = 0);
// Small transfers between the host and the device (counts, per-unit
// results, chain tables) go through pinned memory: a pageable destination
// adds a staging copy inside the runtime.  q_copy(dst, src, n, s): a kernel
// copy (either end device or pinned host memory).  mailbox(c, n): a pinned, coherent region of
// >= n bytes (pinned slot 8), valid until the next mailbox call (one user at
// a time: the context's caller thread).  readback(c, dst, src, n, s): n bytes
// from the device to any host dst through the mailbox, synchronous.
int q_copy(void *dst, const void *src, size_t n, hipStream_t s);
// small transfer into / out of pinned memory: the copy engines
// (hipMemcpyAsync), or with ZT_QCOPY=1 q_copy (A/B: measured slower inside
// the host pipelines, gpurun_out/r06t)
int x_copy(void *dst, const void *src, size_t n, hipStream_t s);
// q_bytes(dst, v, n, s): the n <= 8 low bytes of v (little endian) to device dst, by a kernel
int q_bytes(void *dst, uint64_t v, uint32_t n, hipStream_t s);
int mailbox(DeviceCtx *c, size_t n, void **p);
int readback(DeviceCtx *c, void *h_dst, const void *d_src, size_t n, hipStream_t s);
// Host output buffer the caller frees with zt_free (large ones on huge pages;
// pool = true: from the bounded host output pool, zt_api.cpp); host_release
// is zt_free's second half (back to the pool, or free).  host_direct: [p,
// p + n) lies in a pool buffer registered with HIP, so copies to / from it go
// by DMA without staging.
uint8_t *host_out(size_t n, bool pool = false);
void host_release(void *p);
// host_out_used: the bytes a pooled output actually returns (what zt_free
// registers), when less than requested; host_discard: an output never handed
// out (an error path) freed outright instead of pooled
void host_out_used(void *p, size_t n);
void host_discard(void *p);
bool host_direct(const void *p, size_t n);
// One host allocation for `items` batch outputs (pointers inside it, each
// released by zt_free; reserve >= 1 byte per item so every pointer is
// distinct).  slab_release: true when p lay in a slab (and was released).
uint8_t *slab_out(size_t total, size_t items, bool pool = false);
// device framing of batch members (synth.hip): item k's prefix | body |
// trailer at out + it[k].out_off; trailer 8 = gzip (CRC-32 LE, ISIZE LE),
// 4 = zlib (Adler-32 BE), 0 = none; sums = (crc, adler) per item
struct FrameItem {
  uint64_t body_off;  // in the deflate output
  uint64_t out_off;   // in the framed output
  uint32_t body_len;
  uint32_t isize;
};
int frame_members_dev(const FrameItem *d_items, uint32_t count, const uint8_t *d_prefix, uint32_t plen,
                      uint32_t trailer, const uint8_t *d_body, const uint32_t *d_sums, uint8_t *d_out, hipStream_t s);
bool slab_release(void *p);
// fn(0 .. count-1) over a few host threads when total_bytes is large.
// memcpy into pinned staging with streaming stores (zt_api.cpp)
void copy_to_staging(void *dst, const void *src, size_t n);
void parallel_copy(size_t count, const std::function<void(size_t)> &fn, size_t total_bytes);
// parallel_copy's thread budget on the calling thread (default 8)
void set_copy_threads(size_t k);

// ---- CRC-32 algebra (reflected, P = 0xEDB88320) ------------------------------
// Host and device copies of zlib-style polynomial arithmetic: shifting a raw
// CRC register over n zero bytes is a multiplication by x^(8n) mod P.
#define ZT_CRC_POLY 0xEDB88320u

__host__ __device__ inline uint32_t multmodp(uint32_t a, uint32_t b) {
  uint32_t m = 1u << 31, p = 0;
  for (;;) {
    if (a & m) {
      p ^= b;
      if ((a & (m - 1)) == 0) break;
    }
    m >>= 1;
    b = (b & 1) ? (b >> 1) ^ ZT_CRC_POLY : b >> 1;
  }
  return p;
}

// x^(n * 2^k) mod P from a table of x^(2^k) (period 32)
__host__ __device__ inline uint32_t x2nmodp(const uint32_t *x2n, uint64_t n, unsigned k) {
  uint32_t p = 1u << 31;  // x^0
  while (n) {
    if (n & 1) p = multmodp(x2n[k & 31], p);
    n >>= 1;
    k++;
  }
  return p;
}

// RFC 1951 3.2.5 length / distance code arithmetic, ALU only (table lookups
// indexed by non-provably-uniform values become dependent global loads).
__host__ __device__ __forceinline__ uint32_t len_base(uint32_t ls) {  // ls = symbol - 257, 0..28
  if (ls < 8) return ls + 3;
  if (ls >= 28) return 258;
  uint32_t e = (ls >> 2) - 1;
  return ((4 + (ls & 3)) << e) + 3;
}
__host__ __device__ __forceinline__ uint32_t len_extra(uint32_t ls) {
  return (ls < 8 || ls >= 28) ? 0 : (ls >> 2) - 1;
}
__host__ __device__ __forceinline__ uint32_t dist_base(uint32_t ds) {  // 0..29
  if (ds < 4) return ds + 1;
  uint32_t e = (ds >> 1) - 1;
  return ((2 + (ds & 1)) << e) + 1;
}
__host__ __device__ __forceinline__ uint32_t dist_extra(uint32_t ds) { return ds < 4 ? 0 : (ds >> 1) - 1; }

typedef __attribute__((address_space(1))) const uint8_t g_u8;
typedef __attribute__((address_space(1))) const uint32_t g_u32;

// nibble tables: 16 x 16 for slice-by-8, then 8 x 16 for the multiplication
// by x^(8 * 1024) (checksum.hip's coalesced lane streams)
#define ZT_CRC_NIB_N 384
void crc_host_tables(uint32_t byte_table[256], uint32_t nib[ZT_CRC_NIB_N], uint32_t x2n[32]);
// x^(8 L) mod P for the checksum kernels: [0, 264) unused, then
// ZT_CRC_DIGITS tables of 64 entries x^(8 v 64^d), then per thread of a whole
// segment the shift of its lane stream to the segment end
#define ZT_CRC_DIGITS 6
#define ZT_CRC_DIG_OFF 264
#define ZT_CRC_LANE_OFF (ZT_CRC_DIG_OFF + 64 * ZT_CRC_DIGITS)
#define ZT_CRC_SHIFT_N (ZT_CRC_LANE_OFF + 512)
void crc_shift_tables(const uint32_t x2n[32], uint32_t shift[ZT_CRC_SHIFT_N]);

// ---- launchers (device-resident) ------------------------------------------------
int checksums_dev(DeviceCtx *c, const uint8_t *d_in, size_t n, bool do_crc, bool do_adler, uint32_t crc_in,
                  uint32_t adler_in, uint32_t *d_result /* [2] */, hipStream_t s);
int checksums_batch_dev(DeviceCtx *c, const uint8_t *frame, size_t count, const uint64_t *off, const uint64_t *len,
                        uint32_t *d_result /* [2 count] */, hipStream_t s);
void gzip_header(const zt_gzip_opts *opts, std::vector<uint8_t> &hd);  // container_api.cpp
int current_device();                                                 // zt_api.cpp (this thread's)
std::vector<int> batch_devices();                                     // zt_set_devices, else {current}
// batch deflate (deflate.hip): streams packed at 32 KiB boundaries, one pipeline
size_t deflate_batch_scratch_bytes(const DeviceCtx *c, size_t padded);
int deflate_batch_dev_run(DeviceCtx *c, const uint8_t *d_in, size_t count, const uint64_t *off, const uint64_t *len,
                          int ctype, int level, uint8_t *d_out, uint64_t *out_off, void *scratch_base,
                          size_t scratch_size, hipStream_t s);

// ---- inflate jobs (one stream per wavefront) -----------------------------------
struct InfJob {
  const uint8_t *in;  // whole input array (RawInflate's `input`)
  uint64_t n;         // its length
  uint64_t start;     // RawInflate `index`
  uint8_t *out;       // output buffer (device)
  uint64_t cap;       // output capacity; decoding continues past it, counting only
  int32_t strict;     // stop with 'input buffer is broken' where the reference's EOF test throws
  int32_t resume;     // on an error, still write the output of the blocks that decoded completely
  uint32_t start_bit;      // resume: bits of in[start] already used
  uint32_t hist_len;       // resume: output already produced (match history), <= 32 KiB ...
  const uint8_t *hist;     // ... its bytes (device); `out` receives only the new bytes
  uint32_t stop_first;        // segment decode: first candidate index to test
  const uint64_t *stops;      // sorted segment starts (byte positions in `in`), or null
  uint64_t stop_count;
};

struct InfResult {
  uint64_t out_len;     // bytes produced (may exceed cap)
  uint64_t end_ip;      // reference .ip after decompress
  int32_t status;
  int32_t detail;       // code length / BTYPE for the message
  int32_t strict_fail;  // reference's readBits EOF check would throw
  int32_t stop_idx;     // segment decode: index of the segment start where decoding stopped, -1 at BFINAL
  // resumable decode (zt_inflate_raw_resume): the bit position (relative to
  // `in`) right after the last block that decoded completely and the output
  // length there; the reader's bit position when decoding stopped
  uint64_t blk_bits;
  uint64_t blk_op;
  uint64_t stop_bits;
};

// segment-parallel inflate (restart markers written by deflate); returns 1 when
// the stream has no usable segments (caller decodes it with one wave)
// (*d_out_io null: the output goes to scratch slot 1, returned in *d_out_io;
// a caller-owned output too small for the stream: ZT_E_ARG with *out_len = the
// bytes it needs).  boundary (a byte position, or ~0: none): the decode must
// have a block boundary there -- a unit of the chain starts at it -- or the
// call returns 1 (the pipelined host inflate's certificate that a cut is a
// real block boundary of the whole stream)
int inflate_segments_dev(DeviceCtx *c, const uint8_t *d_in, size_t n, size_t index, uint8_t **d_out_io,
                         size_t out_cap, size_t *out_len, size_t *end_ip, hipStream_t s, uint64_t boundary = ~0ull);


// ---- two-phase token inflate (inflate_tok.hip) ----------------------------------
// phase A: one unit = blocks from one sync point to the next
struct TokJob {
  uint64_t start;       // byte position (relative to `in`) of the unit's first block
  uint64_t tok_off;     // first token slot
  uint32_t tok_cap;     // token capacity
  uint32_t stop_first;  // index of the first sync point after `start`
  uint64_t end;         // end of the unit's input (batch: its stream's end), 0: TokParams::n
};
struct TokResult {
  uint64_t out_len;   // bytes the unit's tokens produce
  uint64_t end_bits;  // bit position after the unit's last block
  uint32_t ntok;
  int32_t status;
  int32_t detail;
  int32_t stop_idx;   // sync point where the unit stopped, -1 at BFINAL
};
struct TokParams {
  const uint8_t *in;
  uint64_t n;
  const uint32_t *order;  // workgroup g decodes unit order[g] (null: unit g)
  const uint64_t *stops;  // sorted sync points
  uint64_t nstops;
  const TokJob *jobs;
  TokResult *res;
  uint32_t *tokens;
  uint32_t count;
  int simt;           // 0: one-lane (scalar) body decode only
  uint64_t *dbg;      // debug: per unit 8 words comparing the SIMT and scalar body decodes, or null
  uint32_t dump_unit; // debug: unit whose first SIMT block dumps per-round lane state after dbg[count * 8]
  uint32_t dump_once;
  // stored payloads of >= kStoredRunMin bytes become three *run tokens*
  // (len << 16 with distance 0, then the payload's input offset, low and high
  // words) whose literal descriptors expand_kernel writes straight from the
  // input; 0: the tokenizer writes a literal token per stored byte
  int run_tokens;
};
constexpr uint32_t kStoredRunMin = 1024;
// phase B: units of the chain, grouped by segment
struct ChainUnit {
  uint64_t tok_off;
  uint64_t out_off;  // absolute output offset
  uint64_t seg_off;  // output offset of the unit's segment
  uint64_t desc_off; // its descriptors (segments start 128-aligned)
  uint32_t ntok;
  uint32_t out_len;
};
struct SegJob {
  uint32_t first, count;  // chain units [first, first + count)
};
// the chain built on the device (inflate_seg.hip chain_kernel); ok == 0: not
// the common case, expand / copy return at once and the host walks the chain
struct ChainInfo {
  int32_t ok;
  uint32_t nseg;
  uint64_t total;       // output bytes
  uint64_t end_bits;    // bit after the last unit's last block
  uint64_t desc_total;  // descriptors
};
struct ResolveParams {
  const uint32_t *tokens;
  const ChainUnit *units;
  const SegJob *segs;
  uint8_t *out;
  uint16_t *desc;        // one descriptor per output byte (expand -> copy)
  int32_t *unit_status;  // expand
  int32_t *seg_status;   // copy
  uint32_t nunits;
  uint32_t nseg;
  int32_t marker;        // expand: segments after the first may reach up to 32 KiB behind their start
  const uint8_t *in;     // expand: the compressed input (payloads of run tokens)
  const ChainInfo *info = nullptr;  // device-built chain: nothing to do unless info->ok; nseg = info->nseg
  const uint32_t *order = nullptr;  // expand: workgroup g takes unit order[g] (null: unit g)
};
int tokenize_units_dev(const TokParams &p, hipStream_t s);
int resolve_segments_dev(const ResolveParams &p, hipStream_t s);
int expand_units_dev(const ResolveParams &p, hipStream_t s);

// ---- general speculative inflate (inflate_gen.hip) ---------------------------------
// A stream without sync points is cut at fixed bit positions; each *unit* is
// decoded by one wave from a start state that is exact (the stream start, a
// redo) or guessed (a candidate block header, a stored block's LEN field, or
// a position inside a block whose header is guessed), up to a stop position.
enum : uint32_t { GK_BLOCK = 0, GK_HUFF = 1, GK_STORED = 2, GK_SHDR = 3, GK_FINAL = 4 };
struct GenState {
  uint64_t pos;     // bit position relative to `in`
  uint64_t hdr;     // GK_HUFF: bit position of the block's header
  uint32_t kind;    // GK_*: a block start, a token start inside a Huffman body,
                    // a byte inside a stored payload, a stored LEN field, the end
  uint32_t rem;     // GK_STORED: payload bytes left
  uint32_t bfinal;  // GK_STORED / GK_SHDR: the block is the last one
  uint32_t pad;
};
struct GenJob {
  GenState st;       // start state
  uint64_t stop;     // the unit ends at the first block / token / payload byte at or after this bit (~0: none)
  uint64_t tok_off;  // token slot
  uint32_t tok_cap;
  uint32_t spec;     // guessed start: record the path's first token starts
};
struct GenResult {
  GenState end;        // state where the unit stopped (GK_FINAL: the stream ended)
  uint64_t out_len;    // bytes its tokens produce
  uint64_t dec_start;  // bit where the recorded token path starts
  uint64_t tab_id;     // tables of that path: its block's header position, or kFixedHdr
  uint64_t out_stop;   // bytes of the tokens before the end state
  uint32_t ntok;       // tokens, including the overlap decoded past the end state
  uint32_t ntok_stop;  // tokens before the end state
  int32_t status;
  int32_t detail;
  uint32_t recorded;   // the token-start bitmap of the first round is valid
  uint32_t tab_final;  // BFINAL of that path's block
  uint32_t tail_ok;    // an overlap past a GK_HUFF end state was decoded (its token starts recorded)
  uint32_t pad;
};
// GenState::hdr of a fixed-code block: every fixed block has the same tables
constexpr uint64_t kFixedHdr = 1ull << 62;
struct GenLink {       // unit k against unit k-1's end state
  uint64_t bytes;      // output bytes of unit k's tokens before the join
  uint64_t prev_bytes; // output bytes of unit k-1's tokens before the join
  uint32_t ok;         // 1: unit k continues unit k-1's path
  uint32_t t;          // unit k's first token on the joint path
  uint32_t prev_cut;   // unit k-1's tokens before the join
  uint32_t pad;
};
struct GenSeg {        // copy segment of the general path
  uint64_t base16;     // its u16 output (byte or window marker) in the staging array
  uint64_t out_off;    // final output offset
  uint64_t len;
};
int inflate_general_dev(DeviceCtx *c, const uint8_t *d_in, size_t n, size_t index, uint8_t **d_out_io,
                        size_t out_cap, size_t *out_len, size_t *end_ip, hipStream_t s);

int inflate_jobs_dev(const InfJob *d_jobs, InfResult *d_res, int count, hipStream_t s);
// one device-resident stream from `index`, output malloc'd (inflate_api.cpp)
int inflate_dev_member(DeviceCtx *c, const uint8_t *d_in, size_t n, size_t index, uint8_t **out, size_t *out_len,
                       size_t *end_ip);
// host -> device copy of n bytes: large buffers through two pinned staging
// chunks (parallel memcpy overlapped with the DMA), small ones directly
int upload(DeviceCtx *c, void *d_dst, const void *h_src, size_t n, hipStream_t s);
// device -> host, the same way; returns after the bytes are in h_dst
int download(DeviceCtx *c, void *h_dst, const void *d_src, size_t n, hipStream_t s);
// Three-stage host pipeline over np pieces, three engines busy at once: piece
// i + 1 crosses PCIe to the device (pinned chunks, stream c->up, one host
// thread) while compute(i) runs on the caller's thread (after piece i's upload
// has landed; it returns the device bytes of its result) and piece i - 1's
// result comes back (stream c->dn, one host thread: straight into a
// registered pool buffer by DMA, else through pinned chunks) to out.base +
// the sum of the earlier results' lengths.
struct PipePiece {
  const void *h_src;  // host bytes of piece i
  void *d_dst;        // where they go on the device
  size_t n;
};
struct PipeOut {
  // host output of `cap` bytes; null: the download stage takes a pooled
  // host_out(cap_fn()) once piece 0 is computed (cap_fn may look at it).  A
  // result that does not fit moves the bytes so far into a larger buffer.  On
  // return -- error or not, every copy finished -- `base` is the caller's.
  uint8_t *base = nullptr;
  size_t cap = 0;
  std::function<size_t()> cap_fn;
  size_t total = 0;  // out: bytes written
  // set by the pipeline for compute(i): drain(j), j < i, makes the compute
  // stream wait until piece j's result has left the device (before compute
  // reuses its device buffer); waits on the host until that copy is issued.
  // Only pieces from drain_from on can be drained: compute sets it (before
  // it returns piece drain_from) when it starts reusing buffers -- an event
  // recorded behind every download cost the inflate pipeline ~3 ms per GiB
  // (gpurun_out/r06u).
  std::function<int(size_t)> drain;
  size_t drain_from = SIZE_MAX;
};
int pipeline_h2d_d2h(DeviceCtx *c, size_t np, const std::function<PipePiece(size_t)> &input,
                     const std::function<int(size_t, const void **d_res, size_t *n_res)> &compute, PipeOut &out);
int inflate_error(int status, int detail);

}  // namespace zt
