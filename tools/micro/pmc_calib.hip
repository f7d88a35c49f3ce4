// pmc_calib.hip -- known-byte kernels for calibrating rocprofv3's FETCH_SIZE /
// WRITE_SIZE on gfx950 (tools/pmc_traffic.py).  Each kernel reads (or
// writes) exactly `n` bytes of a 1 GiB buffer once with one access pattern;
// run under `rocprofv3 --pmc FETCH_SIZE` / `--pmc WRITE_SIZE` and divide the
// counter by n.  Patterns: the ones the engine's kernels use.
//   hipcc -O3 --offload-arch=gfx950 -o tools/micro/pmc_calib tools/micro/pmc_calib.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// 16 bytes per lane, coalesced (match / checksum / gather streams)
__global__ void read16(const u32x4 *in, size_t n16, uint32_t *sink) {
  u32x4 acc = {0, 0, 0, 0};
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x) {
    const u32x4 v = in[i];
    acc ^= v;
  }
  if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) sink[0] = 1;
}
// 4 bytes per lane, coalesced (descriptor / token reads of one dword)
__global__ void read4(const uint32_t *in, size_t n4, uint32_t *sink) {
  uint32_t acc = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x)
    acc ^= in[i];
  if (acc == 0x12345678u) sink[0] = 1;
}
// 2 bytes per lane, coalesced (u16 descriptors)
__global__ void read2(const uint16_t *in, size_t n2, uint32_t *sink) {
  uint32_t acc = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n2; i += (size_t)gridDim.x * blockDim.x)
    acc ^= in[i];
  if (acc == 0x1234u) sink[0] = 1;
}
// LDS-DMA, 4 bytes per lane (parse / copy staging: global_load_lds)
__global__ __launch_bounds__(256) void read_lds_dma(const uint32_t *in, size_t n4, uint32_t *sink) {
  __shared__ uint32_t buf[4][256];
  uint32_t acc = 0;
  const size_t stride = (size_t)gridDim.x * 256;
  int k = 0;
  for (size_t i = blockIdx.x * (size_t)256 + threadIdx.x; i < n4; i += stride, k = (k + 1) & 3) {
    __builtin_amdgcn_global_load_lds(in + i, &buf[k][(threadIdx.x & ~63u)], 4, 0, 0);
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
    acc ^= buf[k][threadIdx.x];
  }
  if (acc == 0x12345678u) sink[0] = 1;
}
// one 64-byte segment per lane (optparse's per-lane group loads: 4 x 16 B of
// a lane's own line, lanes 2 KiB apart)
__global__ void read_lane_lines(const u32x4 *in, size_t n16, uint32_t *sink) {
  u32x4 acc = {0, 0, 0, 0};
  const size_t lanes = (size_t)gridDim.x * blockDim.x;
  const size_t per = n16 / lanes;  // 16-byte words per lane (contiguous)
  const size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  for (size_t j = 0; j + 4 <= per; j += 4) {
    const u32x4 *p = in + t * per + j;
    acc ^= p[0] ^ p[1] ^ p[2] ^ p[3];
  }
  if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) sink[0] = 1;
}
// 16 bytes per lane, coalesced stores
__global__ void write16(u32x4 *out, size_t n16) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x)
    out[i] = u32x4{(uint32_t)i, 1, 2, 3};
}
// 4 bytes per lane, coalesced stores
__global__ void write4(uint32_t *out, size_t n4) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x)
    out[i] = (uint32_t)i;
}

int main() {
  const size_t n = 1ull << 30;
  uint8_t *a, *b;
  uint32_t *sink;
  if (hipMalloc(&a, n) || hipMalloc(&b, n) || hipMalloc(&sink, 64)) return 1;
  (void)hipMemset(a, 1, n);
  (void)hipMemset(b, 0, n);
  (void)hipDeviceSynchronize();
  const int grid = 256 * 8, block = 256;
  // each kernel twice: the second launch is the one to read (cold L2 / MALL for a 1 GiB sweep either way)
  for (int r = 0; r < 2; ++r) {
    read16<<<grid, block>>>((const u32x4 *)a, n / 16, sink);
    read4<<<grid, block>>>((const uint32_t *)a, n / 4, sink);
    read2<<<grid, block>>>((const uint16_t *)a, n / 2, sink);
    read_lds_dma<<<grid, 256>>>((const uint32_t *)a, n / 4, sink);
    read_lane_lines<<<grid, block>>>((const u32x4 *)a, n / 16, sink);
    write16<<<grid, block>>>((u32x4 *)b, n / 16);
    write4<<<grid, block>>>((uint32_t *)b, n / 4);
  }
  if (hipDeviceSynchronize() != hipSuccess) return 2;
  printf("pmc_calib: 7 kernels x 2, %zu bytes each\n", n);
  return 0;
}
