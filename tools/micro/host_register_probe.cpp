// Host-side probe for config C4's pack stage: what registering the callers'
// buffers with HIP costs against packing them into pinned staging.  10 000
// malloc'd buffers of C4's size law (log-uniform 1 KiB .. 1 MiB, seeded),
// split over T threads (T = 1 and 8, as the batch's device threads would):
//   pack:     memcpy of each buffer into one pinned staging buffer
//   register: hipHostRegister + hipHostUnregister of each buffer
// plus one hipHostRegister of a single 1 GiB buffer.  Prints ms and GiB/s.
//   build: hipcc -O2 -o tools/micro/host_register_probe tools/micro/host_register_probe.cpp
#include <hip/hip_runtime.h>

#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <thread>
#include <vector>

static double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main() {
  const int count = 10000;
  std::mt19937_64 rng(1);
  std::uniform_real_distribution<double> u(std::log(1024.0), std::log(1048576.0));
  std::vector<size_t> len(count);
  std::vector<unsigned char *> buf(count);
  size_t total = 0;
  for (int i = 0; i < count; ++i) {
    len[i] = (size_t)std::exp(u(rng));
    buf[i] = (unsigned char *)malloc(len[i]);
    memset(buf[i], i & 0xFF, len[i]);
    total += len[i];
  }
  const double gib = total / 1073741824.0;
  printf("%d buffers, %.3f GiB\n", count, gib);
  void *stage = nullptr;
  if (hipHostMalloc(&stage, total + 4096, hipHostMallocDefault) != hipSuccess) return 1;
  for (int T : {1, 8}) {
    for (int rep = 0; rep < 2; ++rep) {
      std::vector<size_t> off(count + 1, 0);
      for (int i = 0; i < count; ++i) off[i + 1] = off[i] + len[i];
      double t0 = now_ms();
      std::vector<std::thread> th;
      for (int t = 0; t < T; ++t)
        th.emplace_back([&, t] {
          for (int i = t; i < count; i += T) memcpy((unsigned char *)stage + off[i], buf[i], len[i]);
        });
      for (auto &x : th) x.join();
      double pack = now_ms() - t0;
      th.clear();
      std::vector<int> fails(T, 0);
      t0 = now_ms();
      for (int t = 0; t < T; ++t)
        th.emplace_back([&, t] {
          for (int i = t; i < count; i += T)
            if (hipHostRegister(buf[i], len[i], hipHostRegisterDefault) != hipSuccess) ++fails[t];
        });
      for (auto &x : th) x.join();
      double reg = now_ms() - t0;
      th.clear();
      t0 = now_ms();
      for (int t = 0; t < T; ++t)
        th.emplace_back([&, t] {
          for (int i = t; i < count; i += T) (void)hipHostUnregister(buf[i]);
        });
      for (auto &x : th) x.join();
      double unreg = now_ms() - t0;
      int nf = 0;
      for (int f : fails) nf += f;
      printf("threads %d rep %d: pack %.1f ms (%.1f GiB/s) | register %.1f ms (%.1f GiB/s, %.2f us/call, %d failed) "
             "| unregister %.1f ms\n",
             T, rep, pack, gib / (pack / 1e3), reg, gib / (reg / 1e3), reg * 1e3 / count, nf, unreg);
      (void)hipGetLastError();
    }
  }
  const size_t big = 1ull << 30;
  unsigned char *b = (unsigned char *)malloc(big);
  memset(b, 1, big);
  double t0 = now_ms();
  hipError_t e = hipHostRegister(b, big, hipHostRegisterDefault);
  double reg = now_ms() - t0;
  t0 = now_ms();
  (void)hipHostUnregister(b);
  printf("one 1 GiB buffer: register %.1f ms (%s), unregister %.1f ms\n", reg, e == hipSuccess ? "ok" : "failed",
         now_ms() - t0);
  return 0;
}
