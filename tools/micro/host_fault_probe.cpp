// Host-side probe: cost of filling a fresh 1 GiB malloc'd buffer (page
// faults) vs a warm one, with 1 / 4 / 8 threads, with and without
// MADV_HUGEPAGE.  Decides how the host entry points allocate their outputs.
#include <sys/mman.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>
static double fill(unsigned char *dst, const unsigned char *src, size_t n, int nt) {
  auto t0 = std::chrono::steady_clock::now();
  std::vector<std::thread> th;
  size_t per = (n + nt - 1) / nt;
  for (int t = 0; t < nt; ++t) th.emplace_back([=] { size_t a = t * per, b = std::min(n, a + per); memcpy(dst + a, src + a, b - a); });
  for (auto &x : th) x.join();
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}
int main() {
  const size_t n = 1ull << 30;
  unsigned char *src = (unsigned char *)malloc(n);
  memset(src, 7, n);
  for (int huge = 0; huge < 2; ++huge)
    for (int nt : {1, 4, 8, 16}) {
      void *p = nullptr;
      if (posix_memalign(&p, 2u << 20, n)) return 1;
      if (huge) madvise(p, n, MADV_HUGEPAGE);
      double cold = fill((unsigned char *)p, src, n, nt);
      double warm = fill((unsigned char *)p, src, n, nt);
      printf("huge %d threads %2d: fresh %.1f ms, warm %.1f ms\n", huge, nt, cold, warm);
      free(p);
    }
  return 0;
}
