// deflate_api.cpp -- host side of the deflate entry points and the
// device-resident plans (include/zt.h).
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "zt_internal.h"

namespace zt {

size_t deflate_bound_bytes(size_t n);
size_t deflate_segment_bytes();
size_t deflate_scratch_bytes(const DeviceCtx *c, size_t n);
int deflate_dev_run(DeviceCtx *c, const uint8_t *d_in, size_t n, size_t halo, int final_, int ctype, int level,
                    uint8_t *d_out, size_t *out_len, void *scratch_base, size_t scratch_size, hipStream_t s);

static int resolve(const zt_deflate_opts *o, int *ctype, int *level) {
  int ct = o ? o->compression_type : 2;
  int lv = o ? o->level : -1;
  if (ct < 0 || ct > 2) return set_error(ZT_E_INVALID_COMPRESSION_TYPE, "invalid compression type");
  if (lv < 0 || lv > 9) lv = 6;
  if (lv == 0) ct = 0;
  // the reference's `lazy` option asks for deferred matching: use the lazy parse
  if (o && o->lazy > 0 && lv < 4) lv = 4;
  *ctype = ct;
  *level = lv;
  return ZT_OK;
}

static size_t out_bound(int ctype, size_t n) {
  if (ctype == 0) return n + 5 * ((n + 65534) / 65535) + 16;
  return deflate_bound_bytes(n) + (ctype == 1 ? n / 8 + 64 : 0);
}

}  // namespace zt

using namespace zt;

struct zt_deflate_plan {
  int device;
  int ctype, level;
  size_t max_n;
  void *scratch;
  size_t scratch_size;
};

struct zt_inflate_plan {
  int device;
  size_t max_in, max_out;
  void *jobs;
};

extern "C" {

size_t zt_deflate_bound(size_t n) { return out_bound(1, n) + out_bound(0, n); }

int zt_deflate_plan_create(size_t max_n, const zt_deflate_opts *opts, zt_deflate_plan **plan) {
  if (!plan) return set_error(ZT_E_ARG, "null plan");
  DeviceCtx *c;
  ZT_TRY(get_ctx(&c));
  std::lock_guard<std::recursive_mutex> ctx_lock(c->mu);
  int ct, lv;
  ZT_TRY(resolve(opts, &ct, &lv));
  zt_deflate_plan *p = new zt_deflate_plan();
  p->device = c->device;
  p->ctype = ct;
  p->level = lv;
  p->max_n = max_n;
  p->scratch_size = deflate_scratch_bytes(c, max_n);
  hipError_t e = hipMalloc(&p->scratch, p->scratch_size);
  if (e != hipSuccess) {
    delete p;
    return hip_fail(e, "hipMalloc(deflate scratch)");
  }
  *plan = p;
  return ZT_OK;
}

void zt_deflate_plan_destroy(zt_deflate_plan *plan) {
  if (!plan) return;
  if (plan->scratch) (void)hipFree(plan->scratch);
  delete plan;
}

int zt_deflate_dev(zt_deflate_plan *plan, const void *d_in, size_t n, size_t halo, int final_, void *d_out,
                   size_t *out_len, void *stream) {
  if (!plan || !out_len) return set_error(ZT_E_ARG, "null argument");
  if (n > plan->max_n) return set_error(ZT_E_ARG, "input larger than the plan");
  DeviceCtx *c;
  ZT_TRY(get_ctx(&c));
  std::lock_guard<std::recursive_mutex> ctx_lock(c->mu);
  if (plan->device != c->device) return set_error(ZT_E_ARG, "plan belongs to another device (zt_set_device)");
  hipStream_t s = stream ? (hipStream_t)stream : c->stream;
  if (halo > 32768) halo = 32768;
  return deflate_dev_run(c, (const uint8_t *)d_in, n, halo, final_, plan->ctype, plan->level, (uint8_t *)d_out,
                         out_len, plan->scratch, plan->scratch_size, s);
}

// Large host inputs (zt_deflate_raw): PCIe overlapped with the deflate.
// The input is cut into pieces at segment boundaries (restart points, 1 MiB);
// piece i + 1 is uploaded while piece i is deflated and piece i - 1's stream
// comes back (pipeline_h2d_d2h).  A piece deflated with halo 0 and BFINAL
// only on the last one writes exactly its part of the single-call stream (no
// match crosses a restart point; a non-final piece ends with the restart
// marker), so the result is byte-identical to the unpipelined call
// (tests/test_gpu_api_pipeline.py).  Pieces of n / 8 (32-128 MiB) keep >= 2
// match workgroups per CU and bound the fill / drain to one piece.
static constexpr size_t kPipeMin = 64u << 20;

// Piece sizes (whole segments).  From 512 MiB: 64, 128, then 256 MiB pieces
// and the remainder -- a small first piece starts the deflate early, and
// large pieces fill the GPU (a 128 MiB piece's one-wave-per-block kernels
// leave it half empty: 4.1 ms per piece against 3.5 for an eighth of a 1 GiB
// call); 1 GiB: 37.7 -> 34.8 ms (`gpurun_out/r06pc`, `r06pc2`,
// tools/api_deflate_time.py).  Below: n / 8 clamped to 32..128 MiB.  Tuning
// hook ZT_DF_PIECES = a list of MiB "a,b,c" (the last size repeats).
static std::vector<size_t> deflate_pieces(size_t n, size_t seg) {
  static const std::vector<size_t> env = [] {
    std::vector<size_t> v;
    if (const char *e = getenv("ZT_DF_PIECES"))
      for (const char *q = e; *q;) {
        char *end = nullptr;
        const long x = strtol(q, &end, 10);
        if (end == q) break;
        if (x > 0) v.push_back((size_t)x << 20);
        q = *end ? end + 1 : end;
      }
    return v;
  }();
  constexpr size_t MiB = 1u << 20;
  std::vector<size_t> sched = env;
  if (sched.empty()) {
    if (n >= 512 * MiB)
      sched = {64 * MiB, 128 * MiB, 256 * MiB};
    else
      sched = {std::min(std::max(n / 8, 32 * MiB), 128 * MiB)};
  }
  std::vector<size_t> sizes;
  size_t off = 0;
  for (size_t i = 0; off < n; ++i) {
    size_t piece = sched[std::min(i, sched.size() - 1)];
    piece = (piece + seg - 1) / seg * seg;
    piece = std::min(piece, n - off);
    sizes.push_back(piece);
    off += piece;
  }
  return sizes;
}

static int deflate_raw_pipelined(DeviceCtx *c, const uint8_t *in, size_t n, int ct, int lv, uint8_t **out,
                                 size_t *out_len) {
  const std::vector<size_t> sizes = deflate_pieces(n, deflate_segment_bytes());
  const size_t np = sizes.size();
  std::vector<size_t> in_off(np + 1, 0), out_off(np + 1, 0);
  size_t pmax = 0;
  for (size_t i = 0; i < np; ++i) {
    in_off[i + 1] = in_off[i] + sizes[i];
    out_off[i + 1] = out_off[i] + ((out_bound(ct, sizes[i]) + 255) & ~(size_t)255);
    pmax = std::max(pmax, sizes[i]);
  }
  void *d_in, *d_out, *d_scr;
  ZT_TRY(scratch(c, 0, n + 64, &d_in));
  ZT_TRY(scratch(c, 1, out_off[np], &d_out));
  const size_t ss = deflate_scratch_bytes(c, pmax);
  ZT_TRY(scratch(c, 3, ss, &d_scr));
  PipeOut po;
  po.base = host_out(out_off[np], true);
  po.cap = out_off[np];
  if (!po.base) return set_error(ZT_E_NOMEM, "host allocation failed");
  const int rc = pipeline_h2d_d2h(
      c, np,
      [&](size_t i) { return PipePiece{in + in_off[i], (uint8_t *)d_in + in_off[i], sizes[i]}; },
      [&](size_t i, const void **d_res, size_t *n_res) -> int {
        uint8_t *d_o = (uint8_t *)d_out + out_off[i];
        ZT_TRY(deflate_dev_run(c, (const uint8_t *)d_in + in_off[i], sizes[i], 0, i + 1 == np, ct, lv, d_o, n_res,
                               d_scr, ss, c->stream));
        *d_res = d_o;
        return ZT_OK;
      },
      po);
  if (rc) {
    host_discard(po.base);
    return rc;
  }
  host_out_used(po.base, po.total);  // (zt_free registers the stream's pages, not the bound's)
  *out = po.base;
  *out_len = po.total;
  return ZT_OK;
}

int zt_deflate_raw(const uint8_t *in, size_t n, const zt_deflate_opts *opts, uint8_t **out, size_t *out_len) {
  if (!out || !out_len) return set_error(ZT_E_ARG, "null output");
  if (n && !in) return set_error(ZT_E_ARG, "null input");
  DeviceCtx *c;
  ZT_TRY(get_ctx(&c));
  std::lock_guard<std::recursive_mutex> ctx_lock(c->mu);
  int ct, lv;
  ZT_TRY(resolve(opts, &ct, &lv));
  if (ct != 0 && n >= kPipeMin) return deflate_raw_pipelined(c, in, n, ct, lv, out, out_len);
  const size_t ob = out_bound(ct, n);
  void *d_in, *d_out, *d_scr;
  ZT_TRY(scratch(c, 0, n + 64, &d_in));
  ZT_TRY(scratch(c, 1, ob, &d_out));
  const size_t ss = deflate_scratch_bytes(c, n);
  ZT_TRY(scratch(c, 3, ss, &d_scr));
  ZT_TRY(upload(c, d_in, in, n, c->stream));
  size_t len = 0;
  ZT_TRY(deflate_dev_run(c, (const uint8_t *)d_in, n, 0, 1, ct, lv, (uint8_t *)d_out, &len, d_scr, ss, c->stream));
  uint8_t *h = host_out(len, true);
  if (!h) return set_error(ZT_E_NOMEM, "host allocation failed");
  const int rc = download(c, h, d_out, len, c->stream);
  if (rc) {
    zt_free(h);
    return rc;
  }
  *out = h;
  *out_len = len;
  return ZT_OK;
}

int zt_inflate_plan_create(size_t max_in, size_t max_out, zt_inflate_plan **plan) {
  if (!plan) return set_error(ZT_E_ARG, "null plan");
  DeviceCtx *c;
  ZT_TRY(get_ctx(&c));
  std::lock_guard<std::recursive_mutex> ctx_lock(c->mu);
  zt_inflate_plan *p = new zt_inflate_plan();
  p->device = c->device;
  p->max_in = max_in;
  p->max_out = max_out;
  hipError_t e = hipMalloc(&p->jobs, 4096);
  if (e != hipSuccess) {
    delete p;
    return hip_fail(e, "hipMalloc(inflate plan)");
  }
  *plan = p;
  return ZT_OK;
}

void zt_inflate_plan_destroy(zt_inflate_plan *plan) {
  if (!plan) return;
  if (plan->jobs) (void)hipFree(plan->jobs);
  delete plan;
}

int zt_inflate_dev(zt_inflate_plan *plan, const void *d_in, size_t n, void *d_out, size_t out_cap, size_t *out_len,
                   size_t *end_ip, void *stream) {
  if (!plan || !out_len) return set_error(ZT_E_ARG, "null argument");
  DeviceCtx *c;
  ZT_TRY(get_ctx(&c));
  std::lock_guard<std::recursive_mutex> ctx_lock(c->mu);
  if (plan->device != c->device) return set_error(ZT_E_ARG, "plan belongs to another device (zt_set_device)");
  hipStream_t s = stream ? (hipStream_t)stream : c->stream;
  uint8_t *o = (uint8_t *)d_out;
  size_t ol = 0, eip = 0;
  int seg = inflate_segments_dev(c, (const uint8_t *)d_in, n, 0, &o, out_cap, &ol, &eip, s);
  if (seg >= 1) seg = inflate_general_dev(c, (const uint8_t *)d_in, n, 0, &o, out_cap, &ol, &eip, s);
  if (seg < 0) return seg;
  if (seg == 0) {
    *out_len = ol;
    if (end_ip) *end_ip = eip;
    return ZT_OK;
  }
  InfJob job{};
  job.in = (const uint8_t *)d_in;
  job.n = n;
  job.out = (uint8_t *)d_out;
  job.cap = out_cap;
  InfJob *dj = (InfJob *)plan->jobs;
  InfResult *dr = (InfResult *)((uint8_t *)plan->jobs + 256);
  ZT_HIP(hipMemcpyAsync(dj, &job, sizeof job, hipMemcpyHostToDevice, s));
  ZT_TRY(inflate_jobs_dev(dj, dr, 1, s));
  InfResult r;
  ZT_HIP(hipMemcpyAsync(&r, dr, sizeof r, hipMemcpyDeviceToHost, s));
  ZT_HIP(hipStreamSynchronize(s));
  if (r.status) return inflate_error(r.status, r.detail);
  if (r.out_len > out_cap) return set_error(ZT_E_ARG, "output capacity too small");
  *out_len = r.out_len;
  if (end_ip) *end_ip = r.end_ip;
  return ZT_OK;
}

}  // extern "C"
