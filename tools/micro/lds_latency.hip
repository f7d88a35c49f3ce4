// Microbenchmark: dependent-chain latencies seen by a single wave on gfx950
// (LDS pointer chase with readfirstlane, scalar loop, s_memtime rate).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__global__ void chase(uint32_t *out, int iters, int mode) {
  __shared__ uint32_t t[4096];
  for (int i = threadIdx.x; i < 4096; i += blockDim.x) t[i] = (i * 17 + 5) & 4095;
  __syncthreads();
  uint32_t x = 0, acc = 0;
  uint64_t c0 = __builtin_readcyclecounter();
  uint64_t r0 = __builtin_amdgcn_s_memrealtime();
  if (mode == 0) {
    for (int i = 0; i < iters; ++i) x = __builtin_amdgcn_readfirstlane(t[x]);  // uniform chase
  } else if (mode == 1) {
    for (int i = 0; i < iters; ++i) x = t[(x + threadIdx.x) & 4095];  // per-lane chase, no readfirstlane
  } else if (mode == 2) {
    for (int i = 0; i < iters; ++i) { x = __builtin_amdgcn_readfirstlane(x * 1664525u + 1013904223u); acc += x >> 7; }
  } else {
    for (int i = 0; i < iters; ++i) { t[(x + threadIdx.x) & 4095] = x; x = __builtin_amdgcn_readfirstlane(t[x & 4095]) + 1; }
  }
  uint64_t c1 = __builtin_readcyclecounter();
  uint64_t r1 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) {
    out[0] = x + acc;
    out[1] = (uint32_t)(c1 - c0);
    out[2] = (uint32_t)(r1 - r0);
  }
}

int main() {
  uint32_t *d, h[3];
  hipMalloc(&d, 64);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const char *names[4] = {"lds chase + readfirstlane", "lds chase per lane", "salu lcg", "lds write+read chase"};
  for (int mode = 0; mode < 4; ++mode) {
    int iters = 100000;
    chase<<<1, 64>>>(d, 10, mode);
    hipEventRecord(e0);
    chase<<<1, 64>>>(d, iters, mode);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    hipMemcpy(h, d, 12, hipMemcpyDeviceToHost);
    printf("%-28s: %.1f ns/iter wall, %.1f memtime ticks/iter, %.2f realtime(100MHz) ticks/iter -> memtime %.0f MHz\n",
           names[mode], ms * 1e6 / iters, (double)h[1] / iters, (double)h[2] / iters, (double)h[1] / h[2] * 100.0);
  }
  return 0;
}
