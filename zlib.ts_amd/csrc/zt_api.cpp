// zt_api.cpp -- C-ABI entry points (include/zt.h), device contexts, errors.
//
// Every entry point computes on the GPU.  There is deliberately no CPU
// fallback: without a HIP device the calls fail with ZT_E_NO_DEVICE.
#include <immintrin.h>
#include <sys/mman.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <functional>
#include <map>
#include <thread>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <vector>

#include "zt_internal.h"

namespace zt {

static thread_local std::string g_err;
static thread_local int g_dev = 0;

int set_error(int code, const std::string &msg) {
  g_err = msg;
  return code;
}

int hip_fail(hipError_t e, const char *what) {
  char buf[512];
  snprintf(buf, sizeof buf, "HIP error %d (%s) in %s", (int)e, hipGetErrorString(e), what);
  if (e == hipErrorNoDevice || e == hipErrorInvalidDevice) return set_error(ZT_E_NO_DEVICE, buf);
  if (e == hipErrorOutOfMemory) return set_error(ZT_E_NOMEM, buf);
  return set_error(ZT_E_HIP, buf);
}

int timing_begin(DeviceCtx *c, hipStream_t s, int k) {
  if (!c->timing) return ZT_OK;
  ZT_HIP(hipEventRecord(c->ev[2 * k], s));
  return ZT_OK;
}

int timing_end(DeviceCtx *c, hipStream_t s, int k) {
  if (!c->timing) return ZT_OK;
  ZT_HIP(hipEventRecord(c->ev[2 * k + 1], s));
  return ZT_OK;
}

int timing_collect(DeviceCtx *c, double *acc_ms, uint64_t *count, int k) {
  if (!c->timing) return ZT_OK;
  float ms = 0;
  ZT_HIP(hipEventElapsedTime(&ms, c->ev[2 * k], c->ev[2 * k + 1]));
  *acc_ms += ms;
  ++*count;
  return ZT_OK;
}

static std::mutex g_mu;
static std::vector<DeviceCtx *> g_ctx;

// Test-only rehearsal of a multi-GPU node on fewer GPUs: ZT_ALIAS_DEVICES=k
// (read once) makes the library present k logical devices, logical d running
// on HIP device d % (HIP device count) with its own context (streams,
// scratch, pinned staging, host threads) -- what zt_set_devices(mask) spreads
// a batch over.  Unset: logical = HIP devices.
static int hip_count() {
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess) return 0;
  return count;
}
static int alias_count() {
  static const int k = [] {
    const char *e = getenv("ZT_ALIAS_DEVICES");
    const int v = e ? atoi(e) : 0;
    return v > 0 && v <= 64 ? v : 0;
  }();
  return k;
}

int get_ctx(DeviceCtx **out) {
  const int hc = hip_count();
  if (hc <= 0) return set_error(ZT_E_NO_DEVICE, "no HIP device visible (libzt computes on the GPU only)");
  const int count = alias_count() ? alias_count() : hc;
  if (g_dev < 0 || g_dev >= count) return set_error(ZT_E_NO_DEVICE, "invalid device index");
  const int phys = g_dev % hc;
  std::lock_guard<std::mutex> lk(g_mu);
  if (g_ctx.size() < (size_t)count) g_ctx.resize(count, nullptr);
  ZT_HIP(hipSetDevice(phys));
  if (!g_ctx[g_dev]) {
    DeviceCtx *c = new DeviceCtx();
    c->device = g_dev;
    c->phys = phys;
    ZT_HIP(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    ZT_HIP(hipStreamCreateWithFlags(&c->aux, hipStreamNonBlocking));
    ZT_HIP(hipEventCreateWithFlags(&c->aux_ev, hipEventDisableTiming));
    hipDeviceProp_t prop;
    ZT_HIP(hipGetDeviceProperties(&prop, phys));
    c->num_cu = prop.multiProcessorCount;
    uint32_t bt[256], nib[ZT_CRC_NIB_N], x2n[32];
    crc_host_tables(bt, nib, x2n);
    ZT_HIP(hipMalloc(&c->d_crc_nib, sizeof nib));
    ZT_HIP(hipMalloc(&c->d_crc_x2n, sizeof x2n));
    ZT_HIP(hipMemcpy(c->d_crc_nib, nib, sizeof nib, hipMemcpyHostToDevice));
    ZT_HIP(hipMemcpy(c->d_crc_x2n, x2n, sizeof x2n, hipMemcpyHostToDevice));
    uint32_t shift[ZT_CRC_SHIFT_N] = {};
    crc_shift_tables(x2n, shift);
    ZT_HIP(hipMalloc(&c->d_crc_shift, sizeof shift));
    ZT_HIP(hipMemcpy(c->d_crc_shift, shift, sizeof shift, hipMemcpyHostToDevice));
    ZT_HIP(hipMalloc(&c->d_ck_acc, sizeof(CkAcc)));
    ZT_HIP(hipMemset(c->d_ck_acc, 0, sizeof(CkAcc)));
    for (auto &e : c->ev) ZT_HIP(hipEventCreate(&e));
    g_ctx[g_dev] = c;
  }
  *out = g_ctx[g_dev];
  return ZT_OK;
}

int scratch(DeviceCtx *c, int slot, size_t bytes, void **ptr) {
  if (bytes == 0) bytes = 16;
  if (c->buf_size[slot] < bytes) {
    if (c->d_buf[slot]) {
      ZT_HIP(hipDeviceSynchronize());  // any stream may still use it
      ZT_HIP(hipFree(c->d_buf[slot]));
      c->d_buf[slot] = nullptr;
      c->buf_size[slot] = 0;
    }
    size_t sz = bytes + bytes / 4;
    if (const hipError_t e = hipMalloc(&c->d_buf[slot], sz)) {
      c->d_buf[slot] = nullptr;
      (void)hipGetLastError();  // (a caller that falls back must not see it at its next launch check)
      return hip_fail(e, "hipMalloc (scratch)");
    }
    c->buf_size[slot] = sz;
  }
  *ptr = c->d_buf[slot];
  return ZT_OK;
}

// The single-buffer calls' large host outputs (zt_deflate_raw /
// zt_inflate_raw, >= 8 MiB) come from a bounded pool (a caching host
// allocator): zt_free returns such a buffer to the pool -- registered with
// HIP (hipHostRegister) on its first return, a one-time cost of that
// zt_free (~25 ms per GiB, pages past the written output faulted in) -- and
// the next output of a similar size reuses it, so downloads into it and
// uploads from it (a stream handed back to zt_inflate_raw) go by DMA with no
// pinned staging, host memcpy or page faults.  The free buffers the pool
// keeps are bounded by ZT_HOST_POOL_MB (default 4096; 0: no pool, every
// output freshly allocated); zt_release_scratch drops them.  The batch
// calls' slabs (slab_out: the GZip batch's framed members, the batch
// inflate's outputs) come from the pool too -- a slab returns once its last
// item is freed -- so a batch caller in a loop downloads by DMA straight
// into them (C2: 22.7 -> 15.7 ms per 4096 x 64 KiB).
static uint8_t *host_alloc(size_t n) {
  // 2 MiB-aligned and backed by transparent huge pages where the kernel
  // allows it -- 512x fewer first-touch faults while the download fills them
  void *p = nullptr;
  if (posix_memalign(&p, 2u << 20, n)) return nullptr;
  (void)madvise(p, n, MADV_HUGEPAGE);
  return (uint8_t *)p;
}

struct PoolBuf {
  uint8_t *p;
  size_t cap;
  size_t len;      // bytes the current use returns (host_out_used; default: the request)
  size_t hi;       // the most any use returned: the pages ever touched
  size_t reg_len;  // registered prefix (hipHostRegister of [p, p + reg_len)), 0: none
  bool used;
  bool reg_bad;    // registration failed once: not tried again
};
static std::mutex g_pool_mu;
static std::vector<PoolBuf> g_pool;

static size_t pool_limit() {
  static const size_t v = [] {
    const char *e = getenv("ZT_HOST_POOL_MB");
    return e ? (size_t)strtoull(e, nullptr, 10) << 20 : (size_t)4096 << 20;
  }();
  return v;
}

// resident bytes of a free pool buffer: the pages its uses touched
static size_t pool_resident(const PoolBuf &e) { return std::max(e.hi, e.reg_len); }

// free pool buffers beyond the bound, largest first (g_pool_mu held)
static void pool_trim(size_t limit) {
  for (;;) {
    size_t free_bytes = 0, big = SIZE_MAX;
    for (size_t i = 0; i < g_pool.size(); ++i)
      if (!g_pool[i].used) {
        free_bytes += pool_resident(g_pool[i]);
        if (big == SIZE_MAX || pool_resident(g_pool[i]) > pool_resident(g_pool[big])) big = i;
      }
    if (big == SIZE_MAX || (limit && free_bytes <= limit)) return;  // (limit 0: all of them)
    if (g_pool[big].reg_len) (void)hipHostUnregister(g_pool[big].p);
    free(g_pool[big].p);
    g_pool.erase(g_pool.begin() + (long)big);
  }
}

uint8_t *host_out(size_t n, bool pool) {
  if (n < (8u << 20)) return (uint8_t *)malloc(n ? n : 1);
  if (!pool || !pool_limit()) return host_alloc(n);
  {
    std::lock_guard<std::mutex> lk(g_pool_mu);
    size_t best = SIZE_MAX;
    for (size_t i = 0; i < g_pool.size(); ++i) {
      const PoolBuf &e = g_pool[i];
      if (!e.used && e.cap >= n && e.cap / 2 <= n && (best == SIZE_MAX || e.cap < g_pool[best].cap)) best = i;
    }
    if (best != SIZE_MAX) {
      g_pool[best].used = true;
      g_pool[best].len = n;
      return g_pool[best].p;
    }
  }
  uint8_t *p = host_alloc(n);
  if (!p) return nullptr;
  std::lock_guard<std::mutex> lk(g_pool_mu);
  g_pool.push_back(PoolBuf{p, n, n, 0, 0, true, false});
  return p;
}

void host_out_used(void *p, size_t n) {
  std::lock_guard<std::mutex> lk(g_pool_mu);
  for (PoolBuf &e : g_pool)
    if (e.p == p && e.used) e.len = std::min(n, e.cap);
}

// A pool buffer back to the pool (false: p is not one).  The pages its uses
// returned are registered with HIP on the way in -- not its whole capacity
// (a pipelined inflate's buffer is sized for several times its input), and
// outside g_pool_mu (~25 ms per GiB): the buffer stays `used` meanwhile, so
// no other thread takes or trims it, and other threads' host_out / zt_free
// go on.
static bool pool_release(void *p) {
  std::unique_lock<std::mutex> lk(g_pool_mu);
  PoolBuf *e = nullptr;
  for (PoolBuf &x : g_pool)
    if (x.p == p && x.used) e = &x;
  if (!e) return false;
  e->hi = std::max(e->hi, e->len);
  const size_t want = std::min(e->cap, (e->hi + (2u << 20) - 1) & ~(size_t)((2u << 20) - 1));
  if (!e->reg_bad && want > e->reg_len) {
    uint8_t *bp = e->p;
    const size_t old = e->reg_len;
    lk.unlock();
    if (old) (void)hipHostUnregister(bp);
    const bool ok = hipHostRegister(bp, want, hipHostRegisterPortable) == hipSuccess;
    if (!ok) (void)hipGetLastError();
    lk.lock();
    for (PoolBuf &x : g_pool)
      if (x.p == bp) {
        x.reg_len = ok ? want : 0;
        x.reg_bad = !ok;
        x.used = false;
      }
  } else {
    e->used = false;
  }
  pool_trim(pool_limit());
  return true;
}

void host_release(void *p) {
  if (!pool_release(p)) free(p);
}

void host_discard(void *p) {
  if (!p) return;
  {
    std::lock_guard<std::mutex> lk(g_pool_mu);
    for (size_t i = 0; i < g_pool.size(); ++i)
      if (g_pool[i].p == p && g_pool[i].used) {
        if (g_pool[i].reg_len) (void)hipHostUnregister(p);
        g_pool.erase(g_pool.begin() + (long)i);
        break;
      }
  }
  free(p);
}

bool host_direct(const void *p, size_t n) {
  const uint8_t *q = static_cast<const uint8_t *>(p);
  std::lock_guard<std::mutex> lk(g_pool_mu);
  for (const PoolBuf &e : g_pool)
    if (e.used && e.reg_len && q >= e.p && q + n <= e.p + e.reg_len) return true;
  return false;
}

// Batch outputs share one host allocation (a slab, on huge pages when large):
// one allocation and one stream of first-touch faults instead of one per
// item (4096 x 64 KiB outputs: 21 ms of faults in the copy-out).  Each item
// pointer is still released by zt_free; the slab goes with its last item.
struct Slab {
  size_t size;
  size_t refs;
};
static std::mutex g_slab_mu;
static std::map<uintptr_t, Slab> g_slabs;

uint8_t *slab_out(size_t total, size_t items, bool pool) {
  if (total == 0) total = 1;
  uint8_t *b = host_out(total, pool);
  if (!b) return nullptr;
  std::lock_guard<std::mutex> lk(g_slab_mu);
  g_slabs[(uintptr_t)b] = Slab{total, items};
  return b;
}

bool slab_release(void *p) {
  std::lock_guard<std::mutex> lk(g_slab_mu);
  if (g_slabs.empty()) return false;
  auto it = g_slabs.upper_bound((uintptr_t)p);
  if (it == g_slabs.begin()) return false;
  --it;
  if ((uintptr_t)p >= it->first + it->second.size) return false;
  if (--it->second.refs == 0) {
    host_release(reinterpret_cast<void *>(it->first));
    g_slabs.erase(it);
  }
  return true;
}

int pinned(DeviceCtx *c, size_t bytes, void **ptr, int slot) {
  if (bytes == 0) bytes = 16;
  if (c->pinned_size[slot] < bytes) {
    if (c->h_pinned[slot]) {
      ZT_HIP(hipDeviceSynchronize());
      ZT_HIP(hipHostFree(c->h_pinned[slot]));
      c->h_pinned[slot] = nullptr;
      c->pinned_size[slot] = 0;
    }
    size_t sz = bytes + bytes / 4;
    // (slot 1, the inflate metadata, is written and read by q_copy kernels: coherent)
    if (const hipError_t e = hipHostMalloc(&c->h_pinned[slot], sz, slot == 1 ? hipHostMallocCoherent : hipHostMallocDefault)) {
      c->h_pinned[slot] = nullptr;
      (void)hipGetLastError();
      return hip_fail(e, "hipHostMalloc (staging)");
    }
    c->pinned_size[slot] = sz;
  }
  *ptr = c->h_pinned[slot];
  return ZT_OK;
}

int mailbox(DeviceCtx *c, size_t n, void **p) {
  constexpr int kSlot = 8;
  if (n < 4096) n = 4096;
  if (c->pinned_size[kSlot] < n) {
    if (c->h_pinned[kSlot]) {
      ZT_HIP(hipDeviceSynchronize());
      ZT_HIP(hipHostFree(c->h_pinned[kSlot]));
      c->h_pinned[kSlot] = nullptr;
      c->pinned_size[kSlot] = 0;
    }
    const size_t sz = n + n / 4;
    // coherent: the kernels' stores are visible to the host once the stream is synchronized
    if (const hipError_t e = hipHostMalloc(&c->h_pinned[kSlot], sz, hipHostMallocCoherent)) {
      c->h_pinned[kSlot] = nullptr;
      (void)hipGetLastError();
      return hip_fail(e, "hipHostMalloc (mailbox)");
    }
    c->pinned_size[kSlot] = sz;
  }
  *p = c->h_pinned[kSlot];
  return ZT_OK;
}

int x_copy(void *dst, const void *src, size_t n, hipStream_t s) {
  static const bool qc = getenv("ZT_QCOPY") != nullptr;
  if (qc) return q_copy(dst, src, n, s);
  if (n) ZT_HIP(hipMemcpyAsync(dst, src, n, hipMemcpyDefault, s));
  return ZT_OK;
}

int readback(DeviceCtx *c, void *h_dst, const void *d_src, size_t n, hipStream_t s) {
  if (!n) return ZT_OK;
  void *mb;
  ZT_TRY(mailbox(c, n, &mb));
  ZT_TRY(x_copy(mb, d_src, n, s));
  ZT_HIP(hipStreamSynchronize(s));
  memcpy(h_dst, mb, n);
  return ZT_OK;
}

// Large host buffers move through two pinned 32 MiB chunks: the host copy of
// chunk k + 1 (a few threads) overlaps the DMA of chunk k -- pageable
// hipMemcpy stages through the runtime's own small buffers at a fraction of
// the PCIe rate.  Buffers below 8 MiB are copied directly.
static constexpr size_t kXferChunk = 32u << 20;

// (fresh output pages fault in during the copy: 8 threads keep a 32 MiB
// chunk's faults and copy under its DMA time; tools/micro/host_fault_probe)
void copy_to_staging(void *dst, const void *src, size_t n);
static void host_copy(void *dst, const void *src, size_t n) {
  const size_t nt = n >= (16u << 20) ? 8 : n >= (8u << 20) ? 4 : 1;
  if (nt == 1) {
    copy_to_staging(dst, src, n);
    return;
  }
  std::vector<std::thread> th;
  const size_t per = (n + nt - 1) / nt;
  for (size_t t = 0; t < nt; ++t) {
    const size_t a = t * per, b = std::min(n, a + per);
    if (a < b) th.emplace_back([=] { copy_to_staging((uint8_t *)dst + a, (const uint8_t *)src + a, b - a); });
  }
  for (auto &t : th) t.join();
}

static int xfer_setup(DeviceCtx *c, uint8_t **buf) {
  for (int k = 0; k < 2; ++k) {
    void *p;
    ZT_TRY(pinned(c, kXferChunk, &p, 2 + k));
    buf[k] = static_cast<uint8_t *>(p);
    if (!c->xfer_ev[k]) ZT_HIP(hipEventCreateWithFlags(&c->xfer_ev[k], hipEventDisableTiming));
  }
  return ZT_OK;
}

int upload(DeviceCtx *c, void *d_dst, const void *h_src, size_t n, hipStream_t s) {
  if (n < (8u << 20) || host_direct(h_src, n)) {
    if (n) ZT_HIP(hipMemcpyAsync(d_dst, h_src, n, hipMemcpyHostToDevice, s));
    return ZT_OK;
  }
  uint8_t *buf[2];
  ZT_TRY(xfer_setup(c, buf));
  for (size_t off = 0, k = 0; off < n; off += kXferChunk, ++k) {
    const size_t len = std::min(kXferChunk, n - off);
    if (k >= 2) ZT_HIP(hipEventSynchronize(c->xfer_ev[k & 1]));
    host_copy(buf[k & 1], (const uint8_t *)h_src + off, len);
    ZT_HIP(hipMemcpyAsync((uint8_t *)d_dst + off, buf[k & 1], len, hipMemcpyHostToDevice, s));
    ZT_HIP(hipEventRecord(c->xfer_ev[k & 1], s));
  }
  // the staging chunks are reused by the next call: let the last copies land
  ZT_HIP(hipEventSynchronize(c->xfer_ev[0]));
  ZT_HIP(hipEventSynchronize(c->xfer_ev[1]));
  return ZT_OK;
}

int download(DeviceCtx *c, void *h_dst, const void *d_src, size_t n, hipStream_t s) {
  if (n < (8u << 20) || host_direct(h_dst, n)) {
    if (n) ZT_HIP(hipMemcpyAsync(h_dst, d_src, n, hipMemcpyDeviceToHost, s));
    ZT_HIP(hipStreamSynchronize(s));
    return ZT_OK;
  }
  uint8_t *buf[2];
  ZT_TRY(xfer_setup(c, buf));
  const size_t nch = (n + kXferChunk - 1) / kXferChunk;
  auto issue = [&](size_t k) -> int {
    const size_t off = k * kXferChunk, len = std::min(kXferChunk, n - off);
    ZT_HIP(hipMemcpyAsync(buf[k & 1], (const uint8_t *)d_src + off, len, hipMemcpyDeviceToHost, s));
    ZT_HIP(hipEventRecord(c->xfer_ev[k & 1], s));
    return ZT_OK;
  };
  ZT_TRY(issue(0));
  for (size_t k = 0; k < nch; ++k) {
    if (k + 1 < nch) ZT_TRY(issue(k + 1));
    ZT_HIP(hipEventSynchronize(c->xfer_ev[k & 1]));
    const size_t off = k * kXferChunk, len = std::min(kXferChunk, n - off);
    host_copy((uint8_t *)h_dst + off, buf[k & 1], len);
  }
  return ZT_OK;
}

// pipeline_h2d_d2h (zt_internal.h).  Each stage runs in order over the
// pieces; the stages hand pieces on through counters under one mutex, and a
// failing stage stops the others (its error text is re-raised on the
// caller's thread, where zt_last_error_message() reads it).  Every stream the
// pipeline used is drained before it returns, on error paths too: the caller
// may free the output (or the input) as soon as it has the status.
// ZT_PIPE_TIMING=1: per-piece stage timestamps on stderr (measurement only)
static double pt_now() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
static bool pt_on() {
  static const bool on = getenv("ZT_PIPE_TIMING") != nullptr;
  return on;
}
#define PT(...) \
  if (pt_on()) fprintf(stderr, "[pipe %9.3f] " __VA_ARGS__)

int pipeline_h2d_d2h(DeviceCtx *c, size_t np, const std::function<PipePiece(size_t)> &input,
                     const std::function<int(size_t, const void **d_res, size_t *n_res)> &compute, PipeOut &out) {
  const double t_start = pt_now();
  if (!c->up) ZT_HIP(hipStreamCreateWithFlags(&c->up, hipStreamNonBlocking));
  if (!c->dn) ZT_HIP(hipStreamCreateWithFlags(&c->dn, hipStreamNonBlocking));
  uint8_t *stage[4];
  for (int k = 0; k < 4; ++k) {
    void *p;
    ZT_TRY(pinned(c, kXferChunk, &p, 2 + k));
    stage[k] = static_cast<uint8_t *>(p);
    if (!c->xfer_ev[k]) ZT_HIP(hipEventCreateWithFlags(&c->xfer_ev[k], hipEventDisableTiming));
  }
  std::vector<hipEvent_t> landed(np, nullptr), drained(np, nullptr);
  struct EvFree {
    std::vector<hipEvent_t> &v;
    ~EvFree() {
      for (auto e : v)
        if (e) (void)hipEventDestroy(e);
    }
  } ev_free{landed}, ev_free2{drained};
  for (auto &e : landed) ZT_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  for (auto &e : drained) ZT_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));

  std::mutex mu;
  std::condition_variable cv;
  // pieces whose upload is enqueued / whose result is on the device / whose
  // result's copy back is enqueued (with `drained` recorded behind it)
  size_t uploaded = 0, computed = 0, downloaded = 0;
  std::vector<const void *> res(np, nullptr);
  std::vector<size_t> res_n(np, 0);
  int err = 0;
  std::string err_msg;
  auto fail = [&](int rc) {
    std::lock_guard<std::mutex> lk(mu);
    if (!err) {
      err = rc;
      err_msg = zt_last_error_message();
    }
    cv.notify_all();
  };
  auto failed = [&] {
    std::lock_guard<std::mutex> lk(mu);
    return err != 0;
  };
  const int dev = c->phys;
  // stage 1: host -> pinned chunk (host threads) -> device (DMA on c->up)
  auto up_stage = [&]() -> int {
    ZT_HIP(hipSetDevice(dev));
    size_t k = 0;  // chunks issued
    for (size_t i = 0; i < np && !failed(); ++i) {
      const PipePiece pc = input(i);
      if (host_direct(pc.h_src, pc.n)) {  // (a registered pool buffer: DMA from it)
        if (pc.n) ZT_HIP(hipMemcpyAsync(pc.d_dst, pc.h_src, pc.n, hipMemcpyHostToDevice, c->up));
      } else
      for (size_t off = 0; off < pc.n; off += kXferChunk, ++k) {
        const size_t len = std::min(kXferChunk, pc.n - off);
        if (k >= 2) ZT_HIP(hipEventSynchronize(c->xfer_ev[k & 1]));
        host_copy(stage[k & 1], (const uint8_t *)pc.h_src + off, len);
        ZT_HIP(hipMemcpyAsync((uint8_t *)pc.d_dst + off, stage[k & 1], len, hipMemcpyHostToDevice, c->up));
        ZT_HIP(hipEventRecord(c->xfer_ev[k & 1], c->up));
      }
      ZT_HIP(hipEventRecord(landed[i], c->up));
      PT("up %zu issued (%zu B, %s)\n", pt_now() - t_start, i, pc.n, host_direct(pc.h_src, pc.n) ? "direct" : "staged");
      std::lock_guard<std::mutex> lk(mu);
      uploaded = i + 1;
      cv.notify_all();
    }
    return ZT_OK;
  };
  // stage 3: device -> host: straight into a registered pool buffer (DMA on
  // c->dn), else device -> pinned chunk (DMA on c->dn) -> host (host threads)
  uint8_t *base = out.base;
  size_t cap = out.cap, total = 0;
  auto dn_stage = [&]() -> int {
    ZT_HIP(hipSetDevice(dev));
    size_t k = 0;
    for (size_t i = 0; i < np; ++i) {
      {
        std::unique_lock<std::mutex> lk(mu);
        cv.wait(lk, [&] { return computed > i || err; });
        if (err) return ZT_OK;
      }
      const size_t n = res_n[i];
      if (!base) {  // (the output's size estimate may look at piece 0's result)
        cap = std::max(out.cap_fn ? out.cap_fn() : (size_t)0, n);
        base = host_out(cap, true);
        if (!base) return set_error(ZT_E_NOMEM, "host allocation failed");
      }
      PT("dn %zu start (%zu B)\n", pt_now() - t_start, i, n);
      if (total + n > cap) {  // a larger buffer: the bytes so far move over
        PT("dn %zu grows the output %zu -> ...\n", pt_now() - t_start, i, cap);
        const size_t ncap = std::max(2 * cap, total + n + (total + n) / 4);
        uint8_t *nb = host_out(ncap, true);
        if (!nb) return set_error(ZT_E_NOMEM, "host allocation failed");
        ZT_HIP(hipStreamSynchronize(c->dn));
        host_copy(nb, base, total);
        host_discard(base);
        base = nb;
        cap = ncap;
      }
      if (host_direct(base + total, n)) {
        if (n) ZT_HIP(hipMemcpyAsync(base + total, res[i], n, hipMemcpyDeviceToHost, c->dn));
        PT("dn %zu direct\n", pt_now() - t_start, i);
      } else {
        PT("dn %zu staged\n", pt_now() - t_start, i);
        // chunks of this piece: issue k + 1 before copying k out of its staging buffer
        const size_t nch = (n + kXferChunk - 1) / kXferChunk;
        auto issue = [&](size_t j) -> int {
          const size_t off = j * kXferChunk, len = std::min(kXferChunk, n - off);
          ZT_HIP(hipMemcpyAsync(stage[2 + ((k + j) & 1)], (const uint8_t *)res[i] + off, len, hipMemcpyDeviceToHost,
                                c->dn));
          ZT_HIP(hipEventRecord(c->xfer_ev[2 + ((k + j) & 1)], c->dn));
          return ZT_OK;
        };
        if (nch) ZT_TRY(issue(0));
        for (size_t j = 0; j < nch; ++j) {
          if (j + 1 < nch) ZT_TRY(issue(j + 1));
          ZT_HIP(hipEventSynchronize(c->xfer_ev[2 + ((k + j) & 1)]));
          const size_t off = j * kXferChunk, len = std::min(kXferChunk, n - off);
          host_copy(base + total + off, stage[2 + ((k + j) & 1)], len);
        }
        k += nch;
      }
      total += n;
      if (i >= out.drain_from) ZT_HIP(hipEventRecord(drained[i], c->dn));
      std::lock_guard<std::mutex> lk(mu);
      downloaded = i + 1;
      cv.notify_all();
    }
    return ZT_OK;
  };
  out.drain = [&](size_t j) -> int {
    if (j < out.drain_from) return set_error(ZT_E_INTERNAL, "pipeline: drain of a piece before drain_from");
    {
      std::unique_lock<std::mutex> lk(mu);
      cv.wait(lk, [&] { return downloaded > j || err; });
      if (err) return set_error(ZT_E_INTERNAL, "pipeline stopped");
    }
    ZT_HIP(hipStreamWaitEvent(c->stream, drained[j], 0));
    return ZT_OK;
  };
  std::thread tu([&] {
    if (int rc = up_stage()) fail(rc);
  });
  std::thread td([&] {
    if (int rc = dn_stage()) fail(rc);
  });
  // stage 2 on the caller's thread: compute(i) after piece i has landed
  for (size_t i = 0; i < np; ++i) {
    {
      std::unique_lock<std::mutex> lk(mu);
      cv.wait(lk, [&] { return uploaded > i || err; });
      if (err) break;
    }
    int rc = hipStreamWaitEvent(c->stream, landed[i], 0) == hipSuccess ? ZT_OK
                                                                       : set_error(ZT_E_HIP, "hipStreamWaitEvent");
    const void *d = nullptr;
    size_t m = 0;
    PT("compute %zu start\n", pt_now() - t_start, i);
    if (!rc) rc = compute(i, &d, &m);
    PT("compute %zu done (%zu B)\n", pt_now() - t_start, i, m);
    if (rc) {
      fail(rc);
      break;
    }
    std::lock_guard<std::mutex> lk(mu);
    res[i] = d;
    res_n[i] = m;
    computed = i + 1;
    cv.notify_all();
  }
  tu.join();
  td.join();
  PT("joined\n", pt_now() - t_start);
  // nothing may still be copying into the output or out of the input when
  // the caller gets it back (error paths: zt_free / reuse right after)
  const hipError_t e1 = hipStreamSynchronize(c->up), e2 = hipStreamSynchronize(c->dn),
                   e3 = hipStreamSynchronize(c->stream);
  PT("drained\n", pt_now() - t_start);
  out.drain = nullptr;
  out.base = base;
  out.cap = cap;
  out.total = total;
  if (err) {
    (void)hipGetLastError();
    return set_error(err, err_msg);
  }
  if (e1 != hipSuccess) return hip_fail(e1, "pipeline upload stream");
  if (e2 != hipSuccess) return hip_fail(e2, "pipeline download stream");
  if (e3 != hipSuccess) return hip_fail(e3, "pipeline compute stream");
  return ZT_OK;
}

// Copy into staging that only the DMA engine reads back: non-temporal
// (streaming) stores skip the read-for-ownership of every destination line
// and leave the caches to the source -- one read and one write of memory
// traffic per byte instead of two reads and a write, which is what several
// device threads packing at once share (config C4 on 8 GPUs).  AVX2 where
// the host has it, memcpy otherwise; an sfence at the end orders the stores
// before the caller issues the DMA.
__attribute__((target("avx2"))) static void copy_nt_avx2(uint8_t *dst, const uint8_t *src, size_t n) {
  size_t i = 0;
  const size_t head = (32 - ((uintptr_t)dst & 31)) & 31;
  if (head) {
    const size_t h = head < n ? head : n;
    memcpy(dst, src, h);
    i = h;
  }
  for (; i + 128 <= n; i += 128) {
    const __m256i a = _mm256_loadu_si256(reinterpret_cast<const __m256i *>(src + i));
    const __m256i b = _mm256_loadu_si256(reinterpret_cast<const __m256i *>(src + i + 32));
    const __m256i c = _mm256_loadu_si256(reinterpret_cast<const __m256i *>(src + i + 64));
    const __m256i d = _mm256_loadu_si256(reinterpret_cast<const __m256i *>(src + i + 96));
    _mm256_stream_si256(reinterpret_cast<__m256i *>(dst + i), a);
    _mm256_stream_si256(reinterpret_cast<__m256i *>(dst + i + 32), b);
    _mm256_stream_si256(reinterpret_cast<__m256i *>(dst + i + 64), c);
    _mm256_stream_si256(reinterpret_cast<__m256i *>(dst + i + 96), d);
  }
  if (i < n) memcpy(dst + i, src + i, n - i);
  _mm_sfence();
}

void copy_to_staging(void *dst, const void *src, size_t n) {
  static const bool avx2 = __builtin_cpu_supports("avx2") && getenv("ZT_NO_NT_COPY") == nullptr;
  if (avx2 && n >= 4096)
    copy_nt_avx2(static_cast<uint8_t *>(dst), static_cast<const uint8_t *>(src), n);
  else if (n)
    memcpy(dst, src, n);
}

// copy threads of parallel_copy on this thread (the batch's device threads
// split the host's copy threads between them: set_copy_threads)
static thread_local size_t tl_copy_threads = 8;
void set_copy_threads(size_t k) { tl_copy_threads = k < 1 ? 1 : k; }

void parallel_copy(size_t count, const std::function<void(size_t)> &fn, size_t total_bytes) {
  // host memcpy fan-out for the batch paths: one thread per ~8 MiB, at most
  // tl_copy_threads (8 unless a multi-device batch shares them out)
  size_t nt = total_bytes >> 23;
  if (nt > tl_copy_threads) nt = tl_copy_threads;
  if (nt > count) nt = count;
  if (nt < 2) {
    for (size_t i = 0; i < count; ++i) fn(i);
    return;
  }
  std::vector<std::thread> th;
  for (size_t t = 0; t < nt; ++t)
    th.emplace_back([&, t] {
      for (size_t i = t; i < count; i += nt) fn(i);
    });
  for (auto &x : th) x.join();
}

int current_device() { return g_dev; }

static std::mutex g_devs_mu;
static std::vector<int> g_devs;  // zt_set_devices; empty: the calling thread's device

std::vector<int> batch_devices() {
  std::lock_guard<std::mutex> lk(g_devs_mu);
  if (g_devs.empty()) return {g_dev};
  return g_devs;
}

}  // namespace zt

using namespace zt;

extern "C" {

int zt_set_devices(uint64_t mask) {
  const int count = zt_device_count();
  std::vector<int> v;
  for (int d = 0; d < 64; ++d)
    if ((mask >> d) & 1) {
      if (d >= count) return set_error(ZT_E_NO_DEVICE, "invalid device index");
      v.push_back(d);
    }
  std::lock_guard<std::mutex> lk(g_devs_mu);
  g_devs = v;
  return ZT_OK;
}

int zt_device_count(void) {
  const int hc = hip_count();
  return hc > 0 && alias_count() ? alias_count() : hc;
}

int zt_set_device(int device) {
  int count = zt_device_count();
  if (device < 0 || device >= count) return set_error(ZT_E_NO_DEVICE, "invalid device index");
  g_dev = device;
  return ZT_OK;
}

const char *zt_last_error_message(void) { return g_err.c_str(); }

const char *zt_version(void) { return "zlib.ts_amd 0.1 (gfx950)"; }

void zt_free(void *p) {
  if (!p) return;
  if (slab_release(p)) return;
  host_release(p);
}

int zt_dev_checksums(const void *d_in, size_t n, uint32_t crc_in, uint32_t adler_in, uint32_t *crc_out,
                     uint32_t *adler_out, void *stream) {
  DeviceCtx *c;
  ZT_TRY(get_ctx(&c));
  std::lock_guard<std::recursive_mutex> ctx_lock(c->mu);
  hipStream_t s = stream ? (hipStream_t)stream : c->stream;
  if (n == 0) {
    if (crc_out) *crc_out = crc_in;
    if (adler_out) *adler_out = adler_in;
    return ZT_OK;
  }
  void *res;
  ZT_TRY(scratch(c, 2, 16, &res));
  ZT_TRY(checksums_dev(c, (const uint8_t *)d_in, n, crc_out != nullptr, adler_out != nullptr, crc_in, adler_in,
                       (uint32_t *)res, s));
  uint32_t h[2];
  ZT_HIP(hipMemcpyAsync(h, res, sizeof h, hipMemcpyDeviceToHost, s));
  ZT_HIP(hipStreamSynchronize(s));
  if (crc_out) *crc_out = h[0];
  if (adler_out) *adler_out = h[1];
  return ZT_OK;
}

static int checksums_host(const uint8_t *data, size_t len, uint32_t crc_in, uint32_t adler_in, uint32_t *crc_out,
                          uint32_t *adler_out) {
  DeviceCtx *c;
  ZT_TRY(get_ctx(&c));
  std::lock_guard<std::recursive_mutex> ctx_lock(c->mu);
  if (len == 0) {  // the reference returns its inputs untouched (no % 65521)
    if (crc_out) *crc_out = crc_in;
    if (adler_out) *adler_out = adler_in;
    return ZT_OK;
  }
  if (!data) return set_error(ZT_E_ARG, "null data");
  void *d;
  ZT_TRY(scratch(c, 0, len, &d));
  ZT_TRY(upload(c, d, data, len, c->stream));
  return zt_dev_checksums(d, len, crc_in, adler_in, crc_out, adler_out, c->stream);
}

int zt_crc32_update(uint32_t crc, const uint8_t *data, size_t len, uint32_t *out) {
  if (!out) return set_error(ZT_E_ARG, "null out");
  return checksums_host(data, len, crc, 0, out, nullptr);
}

int zt_adler32_update(uint32_t adler, const uint8_t *data, size_t len, uint32_t *out) {
  if (!out) return set_error(ZT_E_ARG, "null out");
  return checksums_host(data, len, 0, adler, nullptr, out);
}

int zt_checksums(const uint8_t *data, size_t len, uint32_t crc_in, uint32_t adler_in, uint32_t *crc_out,
                 uint32_t *adler_out) {
  return checksums_host(data, len, crc_in, adler_in, crc_out, adler_out);
}

int zt_timing_enable(int on) {
  DeviceCtx *c;
  ZT_TRY(get_ctx(&c));
  std::lock_guard<std::recursive_mutex> ctx_lock(c->mu);
  c->timing = on != 0;
  c->times = zt_kernel_times{};
  return ZT_OK;
}

int zt_scratch_bytes(size_t *device_bytes, size_t *pinned_bytes) {
  DeviceCtx *c;
  ZT_TRY(get_ctx(&c));
  std::lock_guard<std::recursive_mutex> ctx_lock(c->mu);
  size_t d = 0, h = 0;
  for (size_t v : c->buf_size) d += v;
  for (size_t v : c->pinned_size) h += v;
  if (device_bytes) *device_bytes = d;
  if (pinned_bytes) *pinned_bytes = h;
  return ZT_OK;
}

int zt_release_scratch(void) {
  DeviceCtx *c;
  ZT_TRY(get_ctx(&c));
  std::lock_guard<std::recursive_mutex> ctx_lock(c->mu);
  ZT_HIP(hipDeviceSynchronize());
  for (int k = 0; k < DeviceCtx::kSlots; ++k) {
    if (c->d_buf[k]) ZT_HIP(hipFree(c->d_buf[k]));
    c->d_buf[k] = nullptr;
    c->buf_size[k] = 0;
  }
  for (int k = 0; k < 10; ++k) {
    if (c->h_pinned[k]) ZT_HIP(hipHostFree(c->h_pinned[k]));
    c->h_pinned[k] = nullptr;
    c->pinned_size[k] = 0;
  }
  std::lock_guard<std::mutex> lk(g_pool_mu);
  pool_trim(0);  // the host output pool's free buffers
  return ZT_OK;
}

int zt_timing_read(zt_kernel_times *out) {
  if (!out) return set_error(ZT_E_ARG, "null output");
  DeviceCtx *c;
  ZT_TRY(get_ctx(&c));
  std::lock_guard<std::recursive_mutex> ctx_lock(c->mu);
  *out = c->times;
  return ZT_OK;
}

}  // extern "C"
