// Does one wave's ds_mskor_rtn_b32 apply conflicting lanes in lane order, so
// that a 16-bit half-word can serve as an exchange target (the match kernel's
// chain heads, if they were u16)?  Lane l writes its id into half (l >> 3) & 1
// of word A(l); the value it gets back must hold, in its half, the id of the
// previous lane with the same (word, half), and the other half must not be
// clobbered by the operation.  Prints the mismatch count.
#include <hip/hip_runtime.h>
#include <cstdio>

__device__ __forceinline__ unsigned mskor(unsigned *p, unsigned clear, unsigned set) {
  unsigned old;
  const unsigned a = (unsigned)(size_t)p;  // LDS address
  asm volatile("ds_mskor_rtn_b32 %0, %1, %2, %3\n\ts_waitcnt lgkmcnt(0)" : "=v"(old) : "v"(a), "v"(clear), "v"(set) : "memory");
  return old;
}

__host__ __device__ int addr_of(int mode, int l) {
  return mode == 0 ? 0 : mode == 1 ? (l & 1) : mode == 2 ? ((l * 7) % 5) : (l >> 4);
}

__global__ void k(unsigned *out, int mode) {
  __shared__ unsigned t[64];
  const int lane = threadIdx.x;
  t[lane] = 0xFFFFFFFFu;
  __syncthreads();
  const int w = addr_of(mode, lane), h = (lane >> 3) & 1;
  const unsigned old = mskor(&t[w], 0xFFFFu << (16 * h), (unsigned)lane << (16 * h));
  __syncthreads();
  out[lane] = (old >> (16 * h)) & 0xFFFFu;
  out[64 + lane] = t[lane];
}

int main() {
  unsigned *d, hbuf[128];
  hipMalloc(&d, 512);
  int bad = 0;
  for (int mode = 0; mode < 4; ++mode) {
    for (int rep = 0; rep < 100; ++rep) {
      hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, mode);
      hipMemcpy(hbuf, d, 512, hipMemcpyDeviceToHost);
      unsigned final_[64];
      for (int i = 0; i < 64; ++i) final_[i] = 0xFFFFFFFFu;
      for (int lane = 0; lane < 64; ++lane) {
        const int w = addr_of(mode, lane), h = (lane >> 3) & 1;
        unsigned want = 0xFFFFu;
        for (int j = lane - 1; j >= 0; --j)
          if (addr_of(mode, j) == w && ((j >> 3) & 1) == h) {
            want = (unsigned)j;
            break;
          }
        if (hbuf[lane] != want) {
          if (bad < 10) printf("mode %d rep %d lane %d got %u want %u\n", mode, rep, lane, hbuf[lane], want);
          ++bad;
        }
        final_[w] = (final_[w] & ~(0xFFFFu << (16 * h))) | ((unsigned)lane << (16 * h));
      }
      for (int i = 0; i < 64; ++i)
        if (hbuf[64 + i] != final_[i]) {
          if (bad < 10) printf("mode %d rep %d word %d final %08x want %08x\n", mode, rep, i, hbuf[64 + i], final_[i]);
          ++bad;
        }
    }
  }
  printf("lane-order mskor: %s (%d mismatches)\n", bad ? "NO" : "yes", bad);
  return 0;
}
