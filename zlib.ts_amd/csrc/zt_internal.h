// zt_internal.h -- shared host/device helpers for libzt (not installed).
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>
#include <string>

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
// One default stream per device plus grow-only scratch buffers, so the
// host-pointer entry points do not hipMalloc on every call.
struct DeviceCtx {
  int device = -1;
  hipStream_t stream = nullptr;
  int num_cu = 0;
  // checksum constants (uploaded once)
  uint32_t *d_crc_nib = nullptr;    // 16 x 16 nibble tables (slice-by-8)
  uint32_t *d_crc_x2n = nullptr;    // x^(2^k) mod P, k = 0..31
  // scratch
  void *d_buf[4] = {nullptr, nullptr, nullptr, nullptr};
  size_t buf_size[4] = {0, 0, 0, 0};
  void *h_pinned = nullptr;
  size_t pinned_size = 0;
};

// Context of the calling thread's current device (created on first use).
int get_ctx(DeviceCtx **out);
// Grow-only device scratch slot `slot` to at least `bytes`.
int scratch(DeviceCtx *c, int slot, size_t bytes, void **ptr);

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

void crc_host_tables(uint32_t byte_table[256], uint32_t nib[256], uint32_t x2n[32]);

// ---- launchers (device-resident) ------------------------------------------------
int checksums_dev(DeviceCtx *c, const uint8_t *d_in, size_t n, bool do_crc, bool do_adler, uint32_t crc_in,
                  uint32_t adler_in, uint32_t *d_result /* [2] */, hipStream_t s);

// ---- inflate jobs (one stream per wavefront) -----------------------------------
struct InfJob {
  const uint8_t *in;  // whole input array (RawInflate's `input`)
  uint64_t n;         // its length
  uint64_t start;     // RawInflate `index`
  uint8_t *out;       // output buffer (device)
  uint64_t cap;       // output capacity; decoding continues past it, counting only
  int32_t strict;     // stop with 'input buffer is broken' where the reference's EOF test throws
  int32_t pad;
};

struct InfResult {
  uint64_t out_len;     // bytes produced (may exceed cap)
  uint64_t end_ip;      // reference .ip after decompress
  int32_t status;
  int32_t detail;       // code length / BTYPE for the message
  int32_t strict_fail;  // reference's readBits EOF check would throw
  int32_t pad;
};

int inflate_jobs_dev(const InfJob *d_jobs, InfResult *d_res, int count, hipStream_t s);
int inflate_error(int status, int detail);

}  // namespace zt
