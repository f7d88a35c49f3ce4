// inflate_api.cpp -- host side of the inflate entry points (include/zt.h).
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "zt_internal.h"

namespace zt {


// Message text of the reference for each status (src/RawInflate.ts).
int inflate_error(int status, int detail) {
  char buf[96];
  switch (status) {
    case ZT_E_INPUT_BROKEN: return set_error(status, "input buffer is broken");
    case ZT_E_INVALID_CODE_LENGTH:
      snprintf(buf, sizeof buf, "invalid code length: %d", detail);
      return set_error(status, buf);
    case ZT_E_UNKNOWN_BTYPE:
      snprintf(buf, sizeof buf, "unknown BTYPE: %d", detail);
      return set_error(status, buf);
    case ZT_E_STORED_LEN: return set_error(status, "invalid uncompressed block header: LEN");
    case ZT_E_STORED_NLEN: return set_error(status, "invalid uncompressed block header: NLEN");
    case ZT_E_INVALID_DISTANCE: return set_error(status, "invalid distance too far back");
    case ZT_E_INVALID_SYMBOL: return set_error(status, "invalid literal/length or distance code");
    case ZT_E_BAD_TREE: return set_error(status, "invalid code lengths set");
    default: return set_error(status, "inflate failed");
  }
}

static size_t align_up(size_t v, size_t a) { return (v + a - 1) / a * a; }

// Decode `count` host streams; outputs are malloc'd.
static int inflate_host_batch(const uint8_t *const *in, const size_t *n, const size_t *index, size_t count,
                              const zt_inflate_opts *opts, uint8_t **out, size_t *out_len, size_t *end_ip,
                              int *status) {
  DeviceCtx *c;
  ZT_TRY(get_ctx(&c));
  const int strict = opts ? opts->ref_strict : 0;
  std::vector<size_t> in_off(count), cap(count);
  size_t in_total = 0;
  for (size_t i = 0; i < count; ++i) {
    in_off[i] = in_total;
    in_total += align_up(n[i] ? n[i] : 1, 256);
    // first guess; exact sizes are known after one pass
    size_t g = n[i] * 4;
    cap[i] = g < 65536 ? 65536 : g;
  }
  void *d_in, *d_jobs, *d_res;
  ZT_TRY(scratch(c, 0, in_total, &d_in));
  ZT_TRY(scratch(c, 2, count * (sizeof(InfJob) + sizeof(InfResult)) + 256, &d_jobs));
  d_res = (uint8_t *)d_jobs + align_up(count * sizeof(InfJob), 256);
  for (size_t i = 0; i < count; ++i)
    if (n[i]) ZT_HIP(hipMemcpyAsync((uint8_t *)d_in + in_off[i], in[i], n[i], hipMemcpyHostToDevice, c->stream));
  std::vector<InfJob> jobs(count);
  std::vector<InfResult> res(count);
  std::vector<size_t> todo(count);
  for (size_t i = 0; i < count; ++i) todo[i] = i;
  for (int pass = 0; pass < 2 && !todo.empty(); ++pass) {
    size_t out_total = 0;
    std::vector<size_t> out_off(todo.size());
    for (size_t k = 0; k < todo.size(); ++k) {
      out_off[k] = out_total;
      out_total += align_up(cap[todo[k]], 256);
    }
    void *d_out;
    ZT_TRY(scratch(c, 1, out_total, &d_out));
    for (size_t k = 0; k < todo.size(); ++k) {
      size_t i = todo[k];
      jobs[k] = InfJob{};
      jobs[k].in = (const uint8_t *)d_in + in_off[i];
      jobs[k].n = n[i];
      jobs[k].start = index ? index[i] : 0;
      jobs[k].out = (uint8_t *)d_out + out_off[k];
      jobs[k].cap = cap[i];
      jobs[k].strict = strict;
    }
    ZT_HIP(hipMemcpyAsync(d_jobs, jobs.data(), todo.size() * sizeof(InfJob), hipMemcpyHostToDevice, c->stream));
    ZT_TRY(inflate_jobs_dev((const InfJob *)d_jobs, (InfResult *)d_res, (int)todo.size(), c->stream));
    std::vector<InfResult> r(todo.size());
    ZT_HIP(hipMemcpyAsync(r.data(), d_res, todo.size() * sizeof(InfResult), hipMemcpyDeviceToHost, c->stream));
    ZT_HIP(hipStreamSynchronize(c->stream));
    std::vector<size_t> again;
    for (size_t k = 0; k < todo.size(); ++k) {
      size_t i = todo[k];
      res[i] = r[k];
      if (r[k].status == ZT_OK && r[k].out_len > cap[i]) {
        cap[i] = r[k].out_len;  // rerun with the exact size
        again.push_back(i);
        continue;
      }
      out[i] = nullptr;
      out_len[i] = 0;
      if (r[k].status == ZT_OK) {
        out[i] = (uint8_t *)malloc(r[k].out_len ? r[k].out_len : 1);
        if (!out[i]) return set_error(ZT_E_NOMEM, "host allocation failed");
        if (r[k].out_len)
          ZT_HIP(hipMemcpyAsync(out[i], (uint8_t *)d_out + out_off[k], r[k].out_len, hipMemcpyDeviceToHost,
                                c->stream));
        out_len[i] = r[k].out_len;
      }
    }
    ZT_HIP(hipStreamSynchronize(c->stream));
    todo.swap(again);
  }
  int first = ZT_OK;
  for (size_t i = 0; i < count; ++i) {
    status[i] = res[i].status;
    if (end_ip) end_ip[i] = res[i].end_ip;
    if (status[i] && first == ZT_OK) first = inflate_error(res[i].status, res[i].detail);
  }
  return first;
}

}  // namespace zt

using namespace zt;

extern "C" {

int zt_inflate_raw(const uint8_t *in, size_t n, size_t index, const zt_inflate_opts *opts, uint8_t **out,
                   size_t *out_len, size_t *end_ip) {
  if (!out || !out_len) return set_error(ZT_E_ARG, "null output");
  if (!(opts && opts->ref_strict) && in && n >= index + (1u << 14)) {
    // large stream: segment-parallel decode when it carries restart points
    DeviceCtx *c;
    ZT_TRY(get_ctx(&c));
    void *d_in;
    ZT_TRY(scratch(c, 0, n, &d_in));
    ZT_HIP(hipMemcpyAsync(d_in, in, n, hipMemcpyHostToDevice, c->stream));
    uint8_t *d_out = nullptr;
    size_t ol = 0, eip = 0;
    const int seg = inflate_segments_dev(c, (const uint8_t *)d_in, n, index, &d_out, 0, &ol, &eip, c->stream);
    if (seg < 0) return seg;
    if (seg == 0) {
      uint8_t *h = (uint8_t *)malloc(ol ? ol : 1);
      if (!h) return set_error(ZT_E_NOMEM, "host allocation failed");
      if (ol) ZT_HIP(hipMemcpyAsync(h, d_out, ol, hipMemcpyDeviceToHost, c->stream));
      ZT_HIP(hipStreamSynchronize(c->stream));
      *out = h;
      *out_len = ol;
      if (end_ip) *end_ip = eip;
      return ZT_OK;
    }
  }
  int st = 0;
  size_t ip = 0;
  const uint8_t *p = in;
  int rc = inflate_host_batch(&p, &n, &index, 1, opts, out, out_len, &ip, &st);
  if (end_ip) *end_ip = ip;
  return rc;
}

int zt_inflate_raw_batch(const uint8_t *const *in, const size_t *n, size_t count, const zt_inflate_opts *opts,
                         uint8_t **out, size_t *out_len, size_t *end_ip, int *status) {
  if (count == 0) return ZT_OK;
  if (!in || !n || !out || !out_len || !status) return set_error(ZT_E_ARG, "null argument");
  return inflate_host_batch(in, n, nullptr, count, opts, out, out_len, end_ip, status);
}

}  // extern "C"
