// Does one wave's ds_wrxchg_rtn_b32 apply conflicting lanes in lane order?
// (the match kernel's chain linking relies on it).  Prints per-lane results.
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(int *out, int mode) {
  __shared__ int t[64];
  const int lane = threadIdx.x;
  if (lane < 64) t[lane] = -1;
  __syncthreads();
  int addr = mode == 0 ? 0 : mode == 1 ? (lane & 1) : mode == 2 ? ((lane * 7) % 5) : (lane >> 4);
  int old = atomicExch(&t[addr], lane);
  __syncthreads();
  out[lane] = old;
  out[64 + lane] = lane < 8 ? t[lane] : 0;
}
int main() {
  int *d, h[128];
  hipMalloc(&d, 512);
  int bad = 0;
  for (int mode = 0; mode < 4; ++mode) {
    for (int rep = 0; rep < 100; ++rep) {
      hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, mode);
      hipMemcpy(h, d, 512, hipMemcpyDeviceToHost);
      // expected: old = previous lane with the same address, else -1
      for (int lane = 0; lane < 64; ++lane) {
        auto A = [&](int l) { return mode == 0 ? 0 : mode == 1 ? (l & 1) : mode == 2 ? ((l * 7) % 5) : (l >> 4); };
        int want = -1;
        for (int j = lane - 1; j >= 0; --j) if (A(j) == A(lane)) { want = j; break; }
        if (h[lane] != want) { if (bad < 10) printf("mode %d rep %d lane %d got %d want %d\n", mode, rep, lane, h[lane], want); ++bad; }
      }
    }
  }
  printf("lane-order xchg: %s (%d mismatches)\n", bad ? "NO" : "yes", bad);
  return 0;
}
