// synth.hip -- synthetic corpora for benchmarks and tests.
// Piece i (64 KiB) of a buffer is generator `kind` seeded with seed + i, so a
// piece equals tools/gen_golden.mjs / oracle zo_gen(kind, seed + i, 65536).
// kind 3 ("mixed") cycles wordsalad / xorshift32 / structured per 4 MiB window.
#include <algorithm>

#include "zt_internal.h"

namespace zt {
namespace {

constexpr uint32_t kPieceBytes = 65536;

__device__ __forceinline__ uint32_t xs32(uint32_t x) {
  x ^= x << 13;
  x ^= x >> 17;
  x ^= x << 5;
  return x;
}

struct WordOut {
  uint32_t *w;
  uint32_t acc = 0, k = 0, i = 0, n;
  __device__ void put(uint32_t b) {
    acc |= b << (8 * k);
    if (++k == 4) {
      w[i >> 2] = acc;
      acc = 0;
      k = 0;
    }
    ++i;
  }
  __device__ void finish(uint8_t *bytes) {
    for (uint32_t j = 0; j < k; ++j) bytes[(i - k) + j] = (uint8_t)(acc >> (8 * j));
  }
};

__global__ __launch_bounds__(64) void synth_kernel(int kind, uint32_t seed, uint8_t *out, uint64_t n,
                                                  uint64_t piece0) {
  const uint64_t lpiece = (uint64_t)blockIdx.x * 64 + threadIdx.x;  // piece of this call's buffer
  const uint64_t lo = lpiece * kPieceBytes;
  if (lo >= n) return;
  const uint64_t piece = piece0 + lpiece;  // piece of the whole (sharded) corpus
  const uint32_t len = (uint32_t)((n - lo) < kPieceBytes ? (n - lo) : kPieceBytes);
  int k = kind;
  if (kind == 3) {
    const int m = (int)((piece >> 6) % 3);
    k = m == 0 ? 1 : m == 1 ? 0 : 2;
  }
  uint32_t x = seed + (uint32_t)piece;
  if (x == 0) x = 0x9E3779B9u;
  WordOut o;
  o.w = reinterpret_cast<uint32_t *>(out + lo);
  o.n = len;
  if (k == 0) {
    for (uint32_t i = 0; i < len; ++i) {
      x = xs32(x);
      o.put(x & 0xFF);
    }
  } else if (k == 1) {
    // 16-word vocabulary, packed: offsets and lengths (the, of, and, deflate, ...)
    const char vocab[] = "theofanddeflatehuffmanwindowstreamblocklz77matchliteralinflategpuwavelanechunk";
    const uint8_t voff[16] = {0, 3, 5, 8, 15, 22, 28, 34, 39, 43, 48, 55, 62, 65, 69, 73};
    const uint8_t vlen[16] = {3, 2, 3, 7, 7, 6, 6, 5, 4, 5, 7, 7, 3, 4, 4, 5};
    while (o.i < len) {
      x = xs32(x);
      const uint32_t w = x & 15;
      for (uint32_t j = 0; j < vlen[w] && o.i < len; ++j) o.put((uint8_t)vocab[voff[w] + j]);
      if (((x >> 4) & 15) == 0) {
        if (o.i < len) o.put('.');
        if (o.i < len) o.put('\n');
      } else if (o.i < len) {
        o.put(' ');
      }
    }
  } else {
    int32_t v = 0;
    for (uint32_t i = 0; i < len; i += 4) {
      x = xs32(x);
      v = (int32_t)((uint32_t)v + (uint32_t)((int32_t)(x & 0xFF) - 128));
      for (uint32_t b = 0; b < 4 && i + b < len; ++b) o.put(((uint32_t)v >> (8 * b)) & 0xFF);
    }
  }
  o.finish(out + lo);
}

// small copies by a kernel (q_copy): dwords when both ends are 4-byte aligned
__global__ __launch_bounds__(256) void q_copy_kernel(uint8_t *__restrict__ dst, const uint8_t *__restrict__ src,
                                                     uint64_t n) {
  const uint64_t t = (uint64_t)blockIdx.x * 256 + threadIdx.x, stride = (uint64_t)gridDim.x * 256;
  if (((reinterpret_cast<uintptr_t>(dst) | reinterpret_cast<uintptr_t>(src)) & 3) == 0) {
    const uint64_t nw = n >> 2;
    for (uint64_t i = t; i < nw; i += stride)
      reinterpret_cast<uint32_t *>(dst)[i] = reinterpret_cast<const uint32_t *>(src)[i];
    for (uint64_t i = (nw << 2) + t; i < n; i += stride) dst[i] = src[i];
  } else {
    for (uint64_t i = t; i < n; i += stride) dst[i] = src[i];
  }
}

__global__ void q_bytes_kernel(uint8_t *dst, uint64_t v, uint32_t n) {
  if (threadIdx.x < n) dst[threadIdx.x] = (uint8_t)(v >> (8 * threadIdx.x));
}

// one workgroup per member: prefix, body, trailer (CRC-32 + ISIZE little
// endian, or Adler-32 big endian)
__global__ __launch_bounds__(256) void frame_members_kernel(const FrameItem *__restrict__ items,
                                                            const uint8_t *__restrict__ prefix, uint32_t plen,
                                                            uint32_t trailer, const uint8_t *__restrict__ body,
                                                            const uint32_t *__restrict__ sums,
                                                            uint8_t *__restrict__ out) {
  const FrameItem it = items[blockIdx.x];
  uint8_t *o = out + it.out_off;
  for (uint32_t i = threadIdx.x; i < plen; i += 256) o[i] = prefix[i];
  const uint8_t *b = body + it.body_off;
  uint8_t *ob = o + plen;
  // (body and destination offsets are arbitrary: dwords read unaligned by
  // byte aligns from the source's aligned words)
  const uint32_t n = it.body_len;
  const uint32_t lead = (uint32_t)((4 - ((uintptr_t)ob & 3)) & 3) < n ? (uint32_t)((4 - ((uintptr_t)ob & 3)) & 3) : n;
  for (uint32_t i = threadIdx.x; i < lead; i += 256) ob[i] = b[i];
  const uint8_t *bs = b + lead;
  uint32_t *od = reinterpret_cast<uint32_t *>(ob + lead);
  const uint32_t nw = (n - lead) / 4;
  const uint32_t sh = (uint32_t)((uintptr_t)bs & 3);
  const uint32_t *sw = reinterpret_cast<const uint32_t *>(bs - sh);
  for (uint32_t w = threadIdx.x; w < nw; w += 256) {
    const uint32_t lo = sw[w], hi = sh ? sw[w + 1] : 0u;
    od[w] = sh ? __builtin_amdgcn_alignbyte(hi, lo, sh) : lo;
  }
  for (uint32_t i = lead + 4 * nw + threadIdx.x; i < n; i += 256) ob[i] = b[i];
  if (threadIdx.x == 0) {
    uint8_t *t = ob + n;
    if (trailer == 8) {
      const uint32_t crc = sums[2 * blockIdx.x];
      for (int k = 0; k < 4; ++k) t[k] = (uint8_t)(crc >> (8 * k));
      for (int k = 0; k < 4; ++k) t[4 + k] = (uint8_t)(it.isize >> (8 * k));
    } else if (trailer == 4) {
      const uint32_t ad = sums[2 * blockIdx.x + 1];
      for (int k = 0; k < 4; ++k) t[k] = (uint8_t)(ad >> (24 - 8 * k));
    }
  }
}

}  // namespace

int frame_members_dev(const FrameItem *d_items, uint32_t count, const uint8_t *d_prefix, uint32_t plen,
                      uint32_t trailer, const uint8_t *d_body, const uint32_t *d_sums, uint8_t *d_out, hipStream_t s) {
  if (!count) return ZT_OK;
  frame_members_kernel<<<count, 256, 0, s>>>(d_items, d_prefix, plen, trailer, d_body, d_sums, d_out);
  ZT_HIP(hipGetLastError());
  return ZT_OK;
}

int q_bytes(void *dst, uint64_t v, uint32_t n, hipStream_t s) {
  if (!n) return ZT_OK;
  q_bytes_kernel<<<1, 64, 0, s>>>(static_cast<uint8_t *>(dst), v, n);
  ZT_HIP(hipGetLastError());
  return ZT_OK;
}

int q_copy(void *dst, const void *src, size_t n, hipStream_t s) {
  if (!n) return ZT_OK;
  const uint64_t blocks = std::min<uint64_t>(1024, (n / 4 + 255) / 256 + 1);
  q_copy_kernel<<<(unsigned)blocks, 256, 0, s>>>(static_cast<uint8_t *>(dst), static_cast<const uint8_t *>(src), n);
  ZT_HIP(hipGetLastError());
  return ZT_OK;
}

}  // namespace zt

using namespace zt;

extern "C" int zt_synth_dev_at(int kind, uint32_t seed, uint64_t piece0, void *d_out, size_t n, void *stream) {
  if (kind < 0 || kind > 3) return set_error(ZT_E_ARG, "unknown generator");
  if (n == 0) return ZT_OK;
  if (!d_out) return set_error(ZT_E_ARG, "null output");
  if (reinterpret_cast<uintptr_t>(d_out) & 3) return set_error(ZT_E_ARG, "output must be 4-byte aligned");
  DeviceCtx *c;
  ZT_TRY(get_ctx(&c));
  std::lock_guard<std::recursive_mutex> ctx_lock(c->mu);
  hipStream_t s = stream ? (hipStream_t)stream : c->stream;
  const uint64_t pieces = (n + kPieceBytes - 1) / kPieceBytes;
  synth_kernel<<<(unsigned)((pieces + 63) / 64), 64, 0, s>>>(kind, seed, static_cast<uint8_t *>(d_out), n, piece0);
  ZT_HIP(hipGetLastError());
  if (!stream) ZT_HIP(hipStreamSynchronize(s));  // library stream: complete before returning
  return ZT_OK;
}

extern "C" int zt_synth_dev(int kind, uint32_t seed, void *d_out, size_t n, void *stream) {
  return zt_synth_dev_at(kind, seed, 0, d_out, n, stream);
}
