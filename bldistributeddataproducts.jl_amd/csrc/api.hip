// api.hip — the extern "C" boundary of libbldp_hip (declared in include/bldp.h).
//
// Argument validation mirrors the reference's error behaviour:
//   * fqavby must divide the selected channel count (Julia reshape in
//     fqav, src/gbtworkerfunctions.jl:18-19 -> DimensionMismatch) => BLDP_EDIM;
//     the same rule is applied to tavby on the time axis;
//   * a window outside the array (h5["data"][idxs...] / dmmap[idxs...],
//     :174,:185 -> BoundsError) => BLDP_EBOUNDS;
//   * everything else that Julia would reject by type or @assert => BLDP_EINVAL.
#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <new>
#include <string>
#include <utility>
#include <vector>

#include "bldp_impl.h"

using namespace bldp;

namespace {

thread_local std::string g_err;

}  // namespace

int bldp::set_error(int code, const char *fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

namespace {

#define fail bldp::set_error

#define HIPCHK(x)                                                                      \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) return fail(BLDP_EHIP, "%s: %s", #x, hipGetErrorString(e_)); \
  } while (0)

// Resolved window: element (c, i, t) at base[off + c*cs + i*ld_i + t*ld_t].
struct Geo {
  int64_t nc, ni, nt;
  int64_t off, cs, ld_i, ld_t;
};

int resolve_window(int64_t nchan, int64_t nif, int64_t ntime, const int64_t *win, Geo *g) {
  if (nchan < 0 || nif < 0 || ntime < 0)
    return fail(BLDP_EINVAL, "negative array dimension (%lld, %lld, %lld)", (long long)nchan,
                (long long)nif, (long long)ntime);
  const int64_t dims[3] = {nchan, nif, ntime};
  int64_t start[3], count[3], step[3];
  for (int ax = 0; ax < 3; ++ax) {
    if (win) {
      start[ax] = win[3 * ax];
      count[ax] = win[3 * ax + 1];
      step[ax] = win[3 * ax + 2];
    } else {
      start[ax] = 0;
      count[ax] = dims[ax];
      step[ax] = 1;
    }
    if (count[ax] < 0) return fail(BLDP_EINVAL, "negative window count on axis %d", ax + 1);
    if (count[ax] > 0) {
      if (step[ax] == 0) return fail(BLDP_EINVAL, "zero window step on axis %d", ax + 1);
      const int64_t last = start[ax] + (count[ax] - 1) * step[ax];
      if (start[ax] < 0 || start[ax] >= dims[ax] || last < 0 || last >= dims[ax])
        return fail(BLDP_EBOUNDS,
                    "BoundsError: window %lld:%lld:%lld (1-based) outside axis %d of size %lld",
                    (long long)(start[ax] + 1), (long long)step[ax], (long long)(last + 1),
                    ax + 1, (long long)dims[ax]);
    }
  }
  g->nc = count[0];
  g->ni = count[1];
  g->nt = count[2];
  const bool empty = g->nc == 0 || g->ni == 0 || g->nt == 0;
  g->off = empty ? 0 : start[0] + nchan * (start[1] + nif * start[2]);
  g->cs = step[0];
  g->ld_i = nchan * step[1];
  g->ld_t = nchan * nif * step[2];
  return BLDP_OK;
}

int resolve_factors(const Geo &g, int64_t fqavby, int64_t tavby, int64_t *F, int64_t *T) {
  *F = fqavby <= 1 ? 1 : fqavby;  // fqav: n <= 1 returns A (src/gbtworkerfunctions.jl:17)
  *T = tavby <= 1 ? 1 : tavby;
  if (g.nc % *F != 0)
    return fail(BLDP_EDIM, "DimensionMismatch: fqavby=%lld does not divide nchan=%lld",
                (long long)*F, (long long)g.nc);
  if (g.nt % *T != 0)
    return fail(BLDP_EDIM, "DimensionMismatch: tavby=%lld does not divide ntime=%lld",
                (long long)*T, (long long)g.nt);
  return BLDP_OK;
}

int num_cus_current() {
  static std::mutex mu;
  static std::map<int, int> cache;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 256;
  std::lock_guard<std::mutex> lk(mu);
  auto it = cache.find(dev);
  if (it != cache.end()) return it->second;
  int n = 256;
  if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    n = 256;
  cache[dev] = n;
  return n;
}

// log2 of the current device's XCD count for the per-XCD tile order
// (hipDeviceAttributeNumberOfXccs: 8 on an MI355X in SPX mode, fewer in the
// compute partitions), 0 when it is 1 or not a power of two.
int xcd_log2_current() {
  static std::mutex mu;
  static std::map<int, int> cache;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 0;
  std::lock_guard<std::mutex> lk(mu);
  auto it = cache.find(dev);
  if (it != cache.end()) return it->second;
  int n = 1, lg = 0;
  if (hipDeviceGetAttribute(&n, hipDeviceAttributeNumberOfXccs, dev) != hipSuccess) n = 1;
  (void)hipGetLastError();
  if (n > 1 && (n & (n - 1)) == 0)
    while ((1 << lg) < n) ++lg;
  cache[dev] = lg;
  return lg;
}

// Library-owned scratch, cached per (device, stream) so that concurrent
// streams never share a buffer.  Host threads sharing one stream (the GBT
// fan-out runs a thread per (worker, file) on torch's current stream) take
// turns: a call holds the entry's lock from the lookup until its last launch
// is queued, so its kernels sit back to back in the stream and the next
// call's kernels run after them.  Growing synchronizes the stream first.
struct Scratch {
  std::mutex mu;
  void *ptr = nullptr;
  size_t bytes = 0;
};
std::mutex g_ws_mu;
std::map<std::pair<int, void *>, Scratch> g_ws;

}  // namespace

int bldp::scratch_lease(hipStream_t s, size_t bytes, ScratchLease *lease) {
  int dev = 0;
  HIPCHK(hipGetDevice(&dev));
  Scratch *w;
  {
    std::lock_guard<std::mutex> lk(g_ws_mu);
    w = &g_ws[{dev, (void *)s}];  // map nodes are stable
  }
  std::unique_lock<std::mutex> hold(w->mu);
  if (w->bytes < bytes) {
    if (w->ptr) {
      HIPCHK(hipStreamSynchronize(s));  // earlier calls on this stream still use it
      HIPCHK(hipFree(w->ptr));
      w->ptr = nullptr;
      w->bytes = 0;
    }
    size_t want = std::max<size_t>(bytes, 1 << 20);
    if (hipMalloc(&w->ptr, want) != hipSuccess) {
      w->ptr = nullptr;
      return fail(BLDP_ENOMEM, "hipMalloc of %zu bytes of scratch failed", want);
    }
    w->bytes = want;
  }
  lease->ptr = w->ptr;
  lease->hold = std::move(hold);
  return BLDP_OK;
}

namespace {
// Staging of bldp_band_reduce_multi_f32's staged banks, one buffer per device
// (kept apart from the per-stream scratch, which the reduces of the same call
// may lease on the same stream).
struct StageBuf {
  std::mutex mu;
  void *ptr = nullptr;
  size_t bytes = 0;
};
std::mutex g_stage_mu;
std::map<int, StageBuf> g_stage;

// The current device's staging buffer of >= bytes, locked into *hold until
// the caller drops the lock (callers synchronize their work before that).
int staging_buffer(int dev, size_t bytes, void **ptr, std::vector<std::unique_lock<std::mutex>> *hold) {
  StageBuf *sb;
  {
    std::lock_guard<std::mutex> lk(g_stage_mu);
    sb = &g_stage[dev];
  }
  std::unique_lock<std::mutex> lk(sb->mu);
  if (sb->bytes < bytes) {
    if (sb->ptr) (void)hipFree(sb->ptr);  // (no work in flight: calls synchronize)
    sb->ptr = nullptr;
    sb->bytes = 0;
    if (hipMalloc(&sb->ptr, bytes) != hipSuccess) {
      sb->ptr = nullptr;
      return fail(BLDP_ENOMEM, "staging allocation of %zu bytes on device %d failed", bytes, dev);
    }
    sb->bytes = bytes;
  }
  *ptr = sb->ptr;
  hold->push_back(std::move(lk));
  return BLDP_OK;
}
}  // namespace

std::vector<int> bldp::scratch_devices() {
  std::lock_guard<std::mutex> lk(g_ws_mu);
  std::vector<int> d;
  for (auto &kv : g_ws) d.push_back(kv.first.first);
  return d;
}

void bldp::scratch_release_all() {
  std::lock_guard<std::mutex> lk(g_ws_mu);
  int prev = -1;
  (void)hipGetDevice(&prev);
  for (auto &kv : g_ws) {
    std::lock_guard<std::mutex> hold(kv.second.mu);  // (callers drained the devices)
    if (kv.second.ptr) {
      (void)hipSetDevice(kv.first.first);
      (void)hipFree(kv.second.ptr);
    }
  }
  g_ws.clear();
  {
    std::lock_guard<std::mutex> lk(g_stage_mu);
    for (auto &kv : g_stage) {
      std::lock_guard<std::mutex> hold(kv.second.mu);
      if (kv.second.ptr) {
        (void)hipSetDevice(kv.first);
        (void)hipFree(kv.second.ptr);
      }
    }
    g_stage.clear();
  }
  if (prev >= 0) (void)hipSetDevice(prev);
}

namespace {


bool aligned16(const void *p) { return ((uintptr_t)p & 15) == 0; }
bool aligned4(const void *p) { return ((uintptr_t)p & 3) == 0; }

bool pitch_ok(const Geo &g) {
  return (g.ni <= 1 || g.ld_i % 4 == 0) && (g.nt <= 1 || g.ld_t % 4 == 0);
}
bool vec_ok(const Geo &g) { return g.cs == 1 && g.off % 4 == 0 && pitch_ok(g); }
// Unit-step windows that start off a 16-byte boundary (or have row pitches
// that are not multiples of 4 floats) on the vector paths (plan option
// "unaligned_vec"): gfx950 executes global_load_dwordx4 at any dword alignment
// (LLVM: unaligned-buffer-access), so the lanes load the window's own float4
// columns and no realignment is needed.  A/B on MI355X
// (profiles/r02/ab_unaligned_vec.json, 8 banks): c0=3 F=64 cfg3 5.42 -> 5.08
// ms, c0=1 F=8 T=1024 cfg4 3.30 -> 2.19 ms, c0=1 F=1 5.92 -> 5.78 ms; but
// c0=1/3 F=1024 4.92 -> 5.12 ms and c0=2 F=2 5.83 -> 6.03 ms (the tile /
// realigning kernels keep those); kurtosis c0=1 cfg4 5.79 -> 2.45 ms, cfg3
// 11.85 -> 6.64 ms (leaf / register paths instead of the two-pass / mid
// ones).  0 = off; 1 = reduce windows where it pays (below); 2 (default) =
// 1 + kurtosis.  (3, every unit-step reduce window: never won; removed in
// round 5.)
// A dword-aligned unit-step reduce window that is not 16-byte aligned goes to
// the vector / narrow paths when that measured faster than the realigning
// kernels, or when the alternative is the scalar path (pitches that are not
// multiples of 4 floats).
bool unaligned_vec_pays(int64_t F, bool rows16) {
  if (!rows16) return true;
  return F == 1 || (F % 4 == 0 && F <= 256);
}

int valid_op(int op) { return op >= BLDP_OP_SUM && op <= BLDP_OP_MIN; }

// Checks, window and plan of a reduce (shared by every reduce entry point and
// by the prepared form): fills *a and *p; *empty when there is nothing to do.
int prepare_reduce(int nbank, const float *const *in, int64_t nchan, int64_t nif, int64_t ntime,
                   const int64_t *win, int64_t fqavby, int64_t tavby, int op, float *out,
                   int64_t out_bank, int64_t out_ld_i, int64_t out_ld_t, bool stitched,
                   bool query, RedArgs *ap, Plan *pp, bool *empty) {
  if (nbank < 1 || nbank > BLDP_MAX_BANKS)
    return fail(BLDP_EINVAL, "nbank=%d outside 1..%d", nbank, BLDP_MAX_BANKS);
  if (!valid_op(op)) return fail(BLDP_EINVAL, "unknown op %d (0=sum 1=mean 2=max 3=min)", op);
  Geo g;
  int rc = resolve_window(nchan, nif, ntime, win, &g);
  if (rc) return rc;
  int64_t F, T;
  rc = resolve_factors(g, fqavby, tavby, &F, &T);
  if (rc) return rc;
  RedArgs &a = *ap;
  a = RedArgs{};
  a.nco = g.nc / F;
  a.ni = g.ni;
  a.nto = g.nt / T;
  a.F = F;
  a.T = T;
  a.nbank = nbank;
  if (stitched) {
    a.out_bank = a.nco;
    a.out_ld_i = nbank * a.nco;
    a.out_ld_t = nbank * a.nco * a.ni;
  } else {
    a.out_bank = out_bank;
    a.out_ld_i = out_ld_i;
    a.out_ld_t = out_ld_t;
  }
  a.in_off = g.off;
  a.in_cs = g.cs;
  a.in_ld_i = g.ld_i;
  a.in_ld_t = g.ld_t;
  a.out = out;
  *empty = a.nco == 0 || a.ni == 0 || a.nto == 0;
  bool rows16 = pitch_ok(g), words = true;
  if (!in) return fail(BLDP_EINVAL, "null input pointer array");
  for (int b = 0; b < nbank; ++b) {
    a.in[b] = in[b];
    rows16 = rows16 && aligned16(a.in[b]);
    words = words && aligned4(a.in[b]);
  }
  const bool aligned = (rows16 && vec_ok(g)) ||
                       (opt(OPT_UNALIGNED_VEC) >= 1 && words && g.cs == 1 &&
                        unaligned_vec_pays(F, rows16));
  *pp = plan_reduce(a, aligned, rows16, words && g.cs == 1, num_cus_current(),
                    xcd_log2_current());
  if (!query) {
    for (int b = 0; b < nbank; ++b)
      if (!in[b] && !*empty) return fail(BLDP_EINVAL, "null input pointer (bank %d)", b);
    if (!out && !*empty) return fail(BLDP_EINVAL, "null output pointer");
  }
  return BLDP_OK;
}

// Queue a prepared reduce on stream s (scratch leased for time-chunk partials).
int run_reduce(RedArgs a, const Plan &p, int op, hipStream_t s) {
  ScratchLease lease;  // held until the launches are queued
  if (p.ws_bytes) {
    int rc = scratch_lease(s, p.ws_bytes, &lease);
    if (rc) return rc;
    a.ws = (float *)lease.ptr;
  }
  hipError_t e = launch_reduce(a, p, op, s);
  if (e != hipSuccess) return fail(BLDP_EHIP, "reduce launch: %s", hipGetErrorString(e));
  return BLDP_OK;
}

int reduce_impl(int nbank, const float *const *in, int64_t nchan, int64_t nif, int64_t ntime,
                const int64_t *win, int64_t fqavby, int64_t tavby, int op, float *out,
                int64_t out_bank, int64_t out_ld_i, int64_t out_ld_t, bool stitched,
                hipStream_t s, int64_t *info) {
  RedArgs a;
  Plan p;
  bool empty = false;
  int rc = prepare_reduce(nbank, in, nchan, nif, ntime, win, fqavby, tavby, op, out, out_bank,
                          out_ld_i, out_ld_t, stitched, info != nullptr, &a, &p, &empty);
  if (rc) return rc;
  if (info) {
    info[0] = p.path;
    info[1] = p.lpg;
    info[2] = p.path == PATH_VEC_ROW ? a.rsplit : a.ts;  // (k_reduce_rows: slices splitting T)
    info[3] = a.k4;
    info[4] = a.nchunk;
    info[5] = p.grid;
    info[6] = (int64_t)p.ws_bytes;
    info[7] = a.vec_out;
    return BLDP_OK;  // plan query only
  }
  if (empty) return BLDP_OK;
  return run_reduce(a, p, op, s);
}

}  // namespace

extern "C" {

int bldp_abi_version(void) { return BLDP_ABI_VERSION; }

int bldp_last_error(char *buf, size_t len) {
  if (!buf || len == 0) return BLDP_EINVAL;
  std::snprintf(buf, len, "%s", g_err.c_str());
  return BLDP_OK;
}

int bldp_device_count(int *n) {
  if (!n) return fail(BLDP_EINVAL, "null pointer");
  HIPCHK(hipGetDeviceCount(n));
  return BLDP_OK;
}

int bldp_plan_option(const char *name, int64_t value, int64_t *previous) {
  if (!name) return fail(BLDP_EINVAL, "null option name");
  const int k = plan_opt_index(name);
  if (k < 0) return fail(BLDP_EINVAL, "unknown plan option '%s'", name);
  if (!plan_opt_valid(k, value)) {
    int64_t lo, hi;
    plan_opt_domain(k, &lo, &hi);
    return fail(BLDP_EINVAL, "plan option '%s' takes %s%lld..%lld or -1 (the default), not %lld",
                name, k == OPT_ROW_SPLIT ? "1, 2 or 4 in " : "", (long long)lo, (long long)hi,
                (long long)value);
  }
  if (previous) *previous = plan_opt_override(k);
  plan_opt_set(k, value < 0 ? -1 : value);
  return BLDP_OK;
}

int bldp_reduce_shape(int64_t nchan, int64_t nif, int64_t ntime, const int64_t *win,
                      int64_t fqavby, int64_t tavby, int64_t out_shape[3]) {
  if (!out_shape) return fail(BLDP_EINVAL, "null out_shape");
  Geo g;
  int rc = resolve_window(nchan, nif, ntime, win, &g);
  if (rc) return rc;
  int64_t F, T;
  rc = resolve_factors(g, fqavby, tavby, &F, &T);
  if (rc) return rc;
  out_shape[0] = g.nc / F;
  out_shape[1] = g.ni;
  out_shape[2] = g.nt / T;
  return BLDP_OK;
}

int bldp_reduce_plan_f32(const float *in, int64_t nchan, int64_t nif, int64_t ntime,
                         const int64_t *win, int64_t fqavby, int64_t tavby, int op,
                         const float *out, int64_t info[8]) {
  if (!info) return fail(BLDP_EINVAL, "null info");
  int64_t sh[3];
  int rc = bldp_reduce_shape(nchan, nif, ntime, win, fqavby, tavby, sh);
  if (rc) return rc;
  const float *ins[1] = {in};
  return reduce_impl(1, ins, nchan, nif, ntime, win, fqavby, tavby, op, (float *)out,
                     sh[0] * sh[1] * sh[2], sh[0], sh[0] * sh[1], false, nullptr, info);
}

int bldp_reduce_f32(const float *in, int64_t nchan, int64_t nif, int64_t ntime,
                    const int64_t *win, int64_t fqavby, int64_t tavby, int op, float *out,
                    void *stream) {
  int64_t sh[3];
  int rc = bldp_reduce_shape(nchan, nif, ntime, win, fqavby, tavby, sh);
  if (rc) return rc;
  const float *ins[1] = {in};
  return reduce_impl(1, ins, nchan, nif, ntime, win, fqavby, tavby, op, out,
                     sh[0] * sh[1] * sh[2], sh[0], sh[0] * sh[1], false, (hipStream_t)stream,
                     nullptr);
}

int bldp_reduce_strided_f32(const float *in, int64_t nchan, int64_t nif, int64_t ntime,
                            const int64_t *win, int64_t fqavby, int64_t tavby, int op,
                            float *out, int64_t out_ld_i, int64_t out_ld_t, void *stream) {
  const float *ins[1] = {in};
  return reduce_impl(1, ins, nchan, nif, ntime, win, fqavby, tavby, op, out, 0, out_ld_i,
                     out_ld_t, false, (hipStream_t)stream, nullptr);
}

int bldp_band_reduce_f32(int nbank, const float *const *in, int64_t nchan, int64_t nif,
                         int64_t ntime, const int64_t *win, int64_t fqavby, int64_t tavby,
                         int op, float *out, void *stream) {
  return reduce_impl(nbank, in, nchan, nif, ntime, win, fqavby, tavby, op, out, 0, 0, 0, true,
                     (hipStream_t)stream, nullptr);
}

// A prepared band reduce: the checks, window, plan and kernel arguments of
// bldp_band_reduce_f32 computed once, so that a launch costs the host nothing
// but the kernel launch itself (a worker re-reducing the same buffers, bench
// loops).
struct bldp_reduce_op {
  // what a launch runs: a Float32 (band) reduce, a typed reduce, a typed
  // getkurtosis, a Float32 getkurtosis (bldp_reduce_prepare /
  // bldp_kurtosis_prepare prepare the last three)
  enum Kind { F32_REDUCE = 0, TYPED_REDUCE, TYPED_KURT, F32_KURT } kind = F32_REDUCE;
  RedArgs a;
  Plan p;
  bldp::TypedArgs t;
  bldp::KurtArgs k;
  double *kout = nullptr;
  int op;
  int dev;
  bool empty;
};

int bldp_band_reduce_prepare_f32(int nbank, const float *const *in, int64_t nchan, int64_t nif,
                                 int64_t ntime, const int64_t *win, int64_t fqavby,
                                 int64_t tavby, int op, float *out, bldp_reduce_op_t *handle) {
  if (!handle) return fail(BLDP_EINVAL, "null handle pointer");
  *handle = nullptr;
  auto *h = new (std::nothrow) bldp_reduce_op{};
  if (!h) return fail(BLDP_ENOMEM, "out of host memory");
  int rc = prepare_reduce(nbank, in, nchan, nif, ntime, win, fqavby, tavby, op, out, 0, 0, 0,
                          true, false, &h->a, &h->p, &h->empty);
  if (rc == BLDP_OK && hipGetDevice(&h->dev) != hipSuccess)
    rc = fail(BLDP_EHIP, "hipGetDevice failed");
  if (rc) {
    delete h;
    return rc;
  }
  h->op = op;
  *handle = h;
  return BLDP_OK;
}

static int kurt_run(KurtArgs &k, double *out, void *workspace, void *stream);

namespace {
// Queue a prepared operation of any kind on s.
int run_prepared(bldp_reduce_op_t h, hipStream_t s) {
  switch (h->kind) {
    case bldp_reduce_op::F32_REDUCE: return run_reduce(h->a, h->p, h->op, s);
    case bldp_reduce_op::TYPED_REDUCE: {
      const hipError_t e = launch_reduce_typed(h->t, h->op, s);
      return e == hipSuccess ? BLDP_OK
                             : fail(BLDP_EHIP, "typed reduce launch: %s", hipGetErrorString(e));
    }
    case bldp_reduce_op::TYPED_KURT: {
      ScratchLease lease;  // time-chunk partial sums (k_kurt_i8), held until queued
      bldp::TypedArgs t = h->t;
      if (const size_t wsb = kurtosis_typed_ws_bytes(t)) {
        const int rc = scratch_lease(s, wsb, &lease);
        if (rc) return rc;
        t.ws = lease.ptr;
        t.ws_bytes = wsb;
      }
      const hipError_t e = launch_kurtosis_typed(t, h->kout, s);
      return e == hipSuccess ? BLDP_OK
                             : fail(BLDP_EHIP, "typed kurtosis launch: %s", hipGetErrorString(e));
    }
    case bldp_reduce_op::F32_KURT: return kurt_run(h->k, h->kout, nullptr, s);
  }
  return fail(BLDP_EINVAL, "bad prepared operation");
}
}  // namespace

int bldp_reduce_launch(bldp_reduce_op_t h, void *stream) {
  if (!h) return fail(BLDP_EINVAL, "null reduce handle");
  if (h->empty) return BLDP_OK;
  int dev = -1;
  if (hipGetDevice(&dev) != hipSuccess || dev != h->dev)
    return fail(BLDP_EINVAL, "reduce handle prepared on device %d, current device %d", h->dev,
                dev);
  return run_prepared(h, (hipStream_t)stream);
}

int bldp_reduce_launch_timed(bldp_reduce_op_t h, void *stream, void *ev_start, void *ev_stop) {
  if (!h) return fail(BLDP_EINVAL, "null reduce handle");
  if (!ev_start || !ev_stop) return fail(BLDP_EINVAL, "null timing event");
  if (h->empty) return BLDP_OK;
  int dev = -1;
  if (hipGetDevice(&dev) != hipSuccess || dev != h->dev)
    return fail(BLDP_EINVAL, "reduce handle prepared on device %d, current device %d", h->dev,
                dev);
  if (h->kind != bldp_reduce_op::F32_REDUCE) {  // events recorded around the launch
    if (hipEventRecord((hipEvent_t)ev_start, (hipStream_t)stream) != hipSuccess)
      return fail(BLDP_EHIP, "hipEventRecord failed");
    const int rc = run_prepared(h, (hipStream_t)stream);
    if (rc) return rc;
    HIPCHK(hipEventRecord((hipEvent_t)ev_stop, (hipStream_t)stream));
    return BLDP_OK;
  }
  set_launch_events((hipEvent_t)ev_start, (hipEvent_t)ev_stop);
  const int rc = run_prepared(h, (hipStream_t)stream);
  set_launch_events(nullptr, nullptr);
  return rc;
}

int bldp_reduce_release(bldp_reduce_op_t h) {
  delete h;
  return BLDP_OK;
}

int bldp_peer_access(int dev, int peer, int *direct) {
  if (!direct) return fail(BLDP_EINVAL, "null pointer");
  *direct = 0;
  int ndev = 0;
  HIPCHK(hipGetDeviceCount(&ndev));
  if (dev < 0 || dev >= ndev || peer < 0 || peer >= ndev)
    return fail(BLDP_EINVAL, "device %d / peer %d not available (%d visible)", dev, peer, ndev);
  if (dev == peer) {
    *direct = 1;
    return BLDP_OK;
  }
  int can = 0;
  if (hipDeviceCanAccessPeer(&can, dev, peer) != hipSuccess || !can) {
    (void)hipGetLastError();
    return BLDP_OK;
  }
  int prev = 0;
  HIPCHK(hipGetDevice(&prev));
  HIPCHK(hipSetDevice(dev));
  const hipError_t pe = hipDeviceEnablePeerAccess(peer, 0);
  (void)hipGetLastError();
  (void)hipSetDevice(prev);
  *direct = pe == hipSuccess || pe == hipErrorPeerAccessAlreadyEnabled;
  return BLDP_OK;
}

int bldp_band_reduce_multi_f32(int nbank, const int *bank_dev, const float *const *in,
                               int64_t nchan, int64_t nif, int64_t ntime, const int64_t *win,
                               int64_t fqavby, int64_t tavby, int op, int root, float *out,
                               unsigned flags) {
  if (nbank < 1 || nbank > BLDP_MAX_BANKS || !bank_dev || !in)
    return fail(BLDP_EINVAL, "bad bank arguments");
  if (flags & ~(BLDP_BAND_STAGED | BLDP_BAND_PEER_STORE))
    return fail(BLDP_EINVAL, "unknown flags 0x%x", flags);
  if ((flags & BLDP_BAND_STAGED) && (flags & BLDP_BAND_PEER_STORE))
    return fail(BLDP_EINVAL, "BLDP_BAND_STAGED and BLDP_BAND_PEER_STORE exclude each other");
  int ndev = 0;
  HIPCHK(hipGetDeviceCount(&ndev));
  if (root < 0 || root >= ndev) return fail(BLDP_EINVAL, "root device %d not available", root);
  for (int b = 0; b < nbank; ++b)
    if (bank_dev[b] < 0 || bank_dev[b] >= ndev)
      return fail(BLDP_EINVAL, "bank %d: device %d not available", b, bank_dev[b]);
  int64_t sh[3];
  int rc = bldp_reduce_shape(nchan, nif, ntime, win, fqavby, tavby, sh);
  if (rc) return rc;
  const int64_t nco = sh[0], ni = sh[1], nto = sh[2];
  if (nco * ni * nto == 0) return BLDP_OK;
  if (!out) return fail(BLDP_EINVAL, "null output pointer");
  const int64_t ld_i = (int64_t)nbank * nco, ld_t = ld_i * ni;
  // BLDP_BAND_STAGED: every bank takes the staged branch (local reduce +
  // strided copy into the root's slot), even on the root device
  const bool force_staged = (flags & BLDP_BAND_STAGED) != 0;
  const bool peer_store = (flags & BLDP_BAND_PEER_STORE) != 0;
  int prev = 0;
  HIPCHK(hipGetDevice(&prev));
  // A device's banks, in bank order, cut into runs whose bank indices step
  // evenly (b0, b0 + s, b0 + 2s, ...): one reduce launch per run, its banks'
  // vcat slots nco * s floats apart.  Contiguous bank-per-device shards (GBT's
  // workers, bench.py's ranks) are one run, i.e. one launch per device.
  struct Run {
    int dev, nb, step;
    int bank[BLDP_MAX_BANKS];
    bool direct;
    size_t stage_off;  // staged runs: floats into the device's staging buffer
  };
  std::vector<Run> runs;
  std::vector<size_t> nstaged(ndev, 0);  // floats of staging per device
  std::vector<hipStream_t> streams(ndev, nullptr);
  const size_t per = (size_t)(nco * ni * nto);
  for (int d = 0; d < ndev && rc == BLDP_OK; ++d) {
    std::vector<int> mine;
    for (int b = 0; b < nbank; ++b)
      if (bank_dev[b] == d) mine.push_back(b);
    if (mine.empty()) continue;
    if ((rc = device_stream(d, &streams[d])) != BLDP_OK) break;
    // the root stores its own slots; another device only with
    // BLDP_BAND_PEER_STORE and peer access (kernel stores over xGMI), else
    // its runs are reduced into staging on the device and DMA-copied
    bool dir = d == root && !force_staged;
    if (!dir && peer_store) {
      int can = 0;
      if (hipDeviceCanAccessPeer(&can, d, root) == hipSuccess && can) {
        if (hipSetDevice(d) != hipSuccess) {
          rc = fail(BLDP_EHIP, "hipSetDevice(%d) failed", d);
          break;
        }
        const hipError_t pe = hipDeviceEnablePeerAccess(root, 0);
        dir = pe == hipSuccess || pe == hipErrorPeerAccessAlreadyEnabled;
      }
      (void)hipGetLastError();
    }
    for (size_t i = 0; i < mine.size();) {
      Run r{};
      r.dev = d;
      r.direct = dir;
      r.bank[0] = mine[i];
      r.nb = 1;
      r.step = i + 1 < mine.size() ? mine[i + 1] - mine[i] : 1;
      while (i + r.nb < mine.size() && mine[i + r.nb] - mine[i + r.nb - 1] == r.step) {
        r.bank[r.nb] = mine[i + r.nb];
        ++r.nb;
      }
      i += r.nb;
      if (!dir) {
        r.stage_off = nstaged[d];
        nstaged[d] += per * r.nb;
      }
      runs.push_back(r);
    }
  }
  // staging: a library-owned buffer per device (no allocation per call once
  // it has grown), held until every launch and copy of this call is done
  // (the call synchronizes before it returns)
  std::vector<std::unique_lock<std::mutex>> hold;
  std::vector<void *> stage(ndev, nullptr);
  for (int d = 0; d < ndev && rc == BLDP_OK; ++d)
    if (nstaged[d]) {
      if (hipSetDevice(d) != hipSuccess) {
        rc = fail(BLDP_EHIP, "hipSetDevice(%d) failed", d);
        break;
      }
      rc = staging_buffer(d, nstaged[d] * sizeof(float), &stage[d], &hold);
    }
  for (const Run &r : runs) {
    if (rc != BLDP_OK) break;
    if (hipSetDevice(r.dev) != hipSuccess) {
      rc = fail(BLDP_EHIP, "hipSetDevice(%d) failed", r.dev);
      break;
    }
    const float *ins[BLDP_MAX_BANKS];
    for (int j = 0; j < r.nb; ++j) ins[j] = in[r.bank[j]];
    if (r.direct) {  // one launch: the run's banks into their slots of the root's product
      rc = reduce_impl(r.nb, ins, nchan, nif, ntime, win, fqavby, tavby, op,
                       out + (int64_t)r.bank[0] * nco, (int64_t)r.step * nco, ld_i, ld_t, false,
                       streams[r.dev], nullptr);
      continue;
    }
    // one launch into staging (the run's banks stitched among themselves),
    // then strided copies into the root's slots: one 2-D copy for a run of
    // neighbouring banks, one per bank otherwise
    float *st = (float *)stage[r.dev] + r.stage_off;
    const int64_t sld_i = (int64_t)r.nb * nco;
    rc = reduce_impl(r.nb, ins, nchan, nif, ntime, win, fqavby, tavby, op, st, nco, sld_i,
                     sld_i * ni, false, streams[r.dev], nullptr);
    const int ncopy = r.step == 1 ? 1 : r.nb;
    const int64_t width = r.step == 1 ? sld_i : nco;
    for (int j = 0; j < ncopy && rc == BLDP_OK; ++j)
      if (hipMemcpy2DAsync(out + (int64_t)r.bank[j] * nco, ld_i * sizeof(float), st + j * nco,
                           sld_i * sizeof(float), width * sizeof(float), (size_t)(ni * nto),
                           hipMemcpyDeviceToDevice, streams[r.dev]) != hipSuccess)
        rc = fail(BLDP_EHIP, "peer copy of bank %d failed", r.bank[j]);
  }
  for (int d = 0; d < ndev; ++d)
    if (streams[d]) {
      (void)hipSetDevice(d);
      if (hipStreamSynchronize(streams[d]) != hipSuccess && rc == BLDP_OK)
        rc = fail(BLDP_EHIP, "device %d failed during the band reduce", d);
    }
  (void)hipSetDevice(prev);
  return rc;
}

int bldp_stitch_f32(int nbank, const float *gathered, int64_t nc, int64_t nif, int64_t ntime,
                    float *out, void *stream) {
  if (nbank < 1 || nbank > BLDP_MAX_BANKS)
    return fail(BLDP_EINVAL, "nbank=%d outside 1..%d", nbank, BLDP_MAX_BANKS);
  if (nc < 0 || nif < 0 || ntime < 0) return fail(BLDP_EINVAL, "negative dimension");
  const int64_t n = nc * nif * ntime;
  if (n > 0 && (!gathered || !out)) return fail(BLDP_EINVAL, "null pointer");
  if (n > 0 && gathered == out) return fail(BLDP_EINVAL, "stitch cannot run in place");
  hipError_t e = launch_stitch(nbank, gathered, nc, nif * ntime, out, (hipStream_t)stream);
  if (e != hipSuccess) return fail(BLDP_EHIP, "stitch launch: %s", hipGetErrorString(e));
  return BLDP_OK;
}

int bldp_despike_f32(float *data, int64_t nchan, int64_t nif, int64_t ntime, int64_t nfpc,
                     void *stream) {
  if (nchan < 0 || nif < 0 || ntime < 0) return fail(BLDP_EINVAL, "negative dimension");
  // spike = nfpc÷2 + 1 (1-based, src/gbt.jl:102); spike-1 must be a valid index
  if (nfpc < 2) return fail(BLDP_EBOUNDS, "BoundsError: nfpc=%lld < 2", (long long)nfpc);
  const int64_t sp = nfpc / 2;  // 0-based spike bin
  const int64_t nspike = nchan > sp ? (nchan - sp + nfpc - 1) / nfpc : 0;
  const int64_t nsrc = nchan > sp - 1 ? (nchan - (sp - 1) + nfpc - 1) / nfpc : 0;
  if (nspike != nsrc)  // d[spike:nfpc:end] .= d[spike-1:nfpc:end] length mismatch
    return fail(BLDP_EDIM,
                "DimensionMismatch: %lld spike bins vs %lld source bins (nchan=%lld, nfpc=%lld)",
                (long long)nspike, (long long)nsrc, (long long)nchan, (long long)nfpc);
  if (nspike * nif * ntime > 0 && !data) return fail(BLDP_EINVAL, "null pointer");
  hipError_t e = launch_despike(data, nchan, nif * ntime, nfpc, nspike, (hipStream_t)stream);
  if (e != hipSuccess) return fail(BLDP_EHIP, "despike launch: %s", hipGetErrorString(e));
  return BLDP_OK;
}

static int kurt_setup(int nbank, const float *const *in, int64_t nchan, int64_t nif,
                      int64_t ntime, const int64_t *win, KurtArgs *k) {
  if (nbank < 1 || nbank > BLDP_MAX_BANKS)
    return fail(BLDP_EINVAL, "nbank=%d outside 1..%d", nbank, BLDP_MAX_BANKS);
  Geo g;
  int rc = resolve_window(nchan, nif, ntime, win, &g);
  if (rc) return rc;
  *k = KurtArgs{};
  k->nbank = nbank;
  bool aligned = true, words = true;
  for (int b = 0; b < nbank; ++b) {
    k->in[b] = in ? in[b] : nullptr;
    aligned = aligned && aligned16(k->in[b]);
    words = words && aligned4(k->in[b]);
  }
  k->in_off = g.off;
  k->in_cs = g.cs;
  k->in_ld_i = g.ld_i;
  k->in_ld_t = g.ld_t;
  k->nc = g.nc;
  k->ni = g.ni;
  k->nt = g.nt;
  k->nrow = (int64_t)nbank * g.ni;
  k->rows16 = vec_ok(g) && g.nc % 4 == 0 && aligned;
  k->vec = opt(OPT_UNALIGNED_VEC) >= 2 ? (g.cs == 1 && g.nc % 4 == 0 && words) : k->rows16;
  plan_kurtosis(*k, num_cus_current());
  return BLDP_OK;
}

static int kurt_run(KurtArgs &k, double *out, void *workspace, void *stream) {
  if (k.nc * k.nrow == 0) return BLDP_OK;
  if (kurtosis_max_grid(k) > INT32_MAX)
    return fail(BLDP_EINVAL, "kurtosis window too large for one launch");
  for (int b = 0; b < k.nbank; ++b)
    if (!k.in[b] && k.nt > 0) return fail(BLDP_EINVAL, "null input pointer (bank %d)", b);
  if (!out) return fail(BLDP_EINVAL, "null output pointer");
  k.out = out;
  hipStream_t s = (hipStream_t)stream;
  void *ws = workspace;
  ScratchLease lease;  // held until the launches are queued
  if (!ws) {
    int rc = scratch_lease(s, kurtosis_ws_bytes(k), &lease);
    if (rc) return rc;
    ws = lease.ptr;
  }
  hipError_t e = launch_kurtosis(k, (char *)ws, s);
  if (e != hipSuccess) return fail(BLDP_EHIP, "kurtosis launch: %s", hipGetErrorString(e));
  return BLDP_OK;
}

size_t bldp_kurtosis_workspace_size(int64_t nchan, int64_t nif, int64_t ntime,
                                    const int64_t *win) {
  KurtArgs k;
  const float *none[1] = {nullptr};
  if (kurt_setup(1, none, nchan, nif, ntime, win, &k)) return 0;
  // enough for either plan: the path depends on the pointer's alignment
  k.vec = 1;
  const size_t a = kurtosis_ws_bytes(k);
  k.vec = 0;
  return std::max(a, kurtosis_ws_bytes(k));
}

int bldp_kurtosis_plan_f32(const float *in, int64_t nchan, int64_t nif, int64_t ntime,
                           const int64_t *win, int64_t info[4]) {
  if (!info) return fail(BLDP_EINVAL, "null info");
  KurtArgs k;
  const float *ins[1] = {in};
  int rc = kurt_setup(1, ins, nchan, nif, ntime, win, &k);
  if (rc) return rc;
  info[0] = kurtosis_path(k);
  info[1] = k.K;
  info[2] = k.nslot;
  info[3] = (int64_t)kurtosis_ws_bytes(k);
  return BLDP_OK;
}

int bldp_kurtosis_f32(const float *in, int64_t nchan, int64_t nif, int64_t ntime,
                      const int64_t *win, double *out, void *workspace, void *stream) {
  KurtArgs k;
  const float *ins[1] = {in};
  int rc = kurt_setup(1, ins, nchan, nif, ntime, win, &k);
  if (rc) return rc;
  return kurt_run(k, out, workspace, stream);
}

int bldp_band_kurtosis_f32(int nbank, const float *const *in, int64_t nchan, int64_t nif,
                           int64_t ntime, const int64_t *win, double *out, void *stream) {
  if (!in) return fail(BLDP_EINVAL, "null input pointer array");
  KurtArgs k;
  int rc = kurt_setup(nbank, in, nchan, nif, ntime, win, &k);
  if (rc) return rc;
  return kurt_run(k, out, nullptr, stream);
}

int bldp_reduce_out_dtype(int dtype, int op) {
  const int d = typed_out_dtype(dtype, op);
  if (d < 0) return fail(BLDP_EINVAL, "unknown element type %d or op %d", dtype, op);
  return d;
}

}  // extern "C"

namespace {
// The TypedArgs of a typed reduce (bldp_reduce_strided's checks); *empty when
// there is nothing to do.
int typed_reduce_args(int dtype, const void *in, int64_t nchan, int64_t nif, int64_t ntime,
                      const int64_t *win, int64_t fqavby, int64_t tavby, int op, void *out,
                      int64_t out_ld_i, int64_t out_ld_t, TypedArgs *ap, bool *empty) {
  if (!dtype_size(dtype)) return fail(BLDP_EINVAL, "unknown element type %d", dtype);
  if (!valid_op(op)) return fail(BLDP_EINVAL, "unknown op %d (0=sum 1=mean 2=max 3=min)", op);
  Geo g;
  int rc = resolve_window(nchan, nif, ntime, win, &g);
  if (rc) return rc;
  int64_t F, T;
  rc = resolve_factors(g, fqavby, tavby, &F, &T);
  if (rc) return rc;
  TypedArgs &a = *ap;
  a = TypedArgs{};
  a.dtype = dtype;
  a.nbank = 1;
  a.in[0] = in;
  a.out = out;
  a.out_ld_i = out_ld_i;
  a.out_ld_t = out_ld_t;
  a.in_off = g.off;
  a.in_cs = g.cs;
  a.in_ld_i = g.ld_i;
  a.in_ld_t = g.ld_t;
  a.nco = g.nc / F;
  a.ni = g.ni;
  a.nto = g.nt / T;
  a.F = F;
  a.T = T;
  a.num_cus = num_cus_current();
  *empty = a.nco * a.ni * a.nto == 0;
  if (*empty) return BLDP_OK;
  if (!in || !out) return fail(BLDP_EINVAL, "null pointer");
  return BLDP_OK;
}

// The TypedArgs of a typed getkurtosis (bldp_kurtosis's checks).
int typed_kurt_args(int dtype, const void *in, int64_t nchan, int64_t nif, int64_t ntime,
                    const int64_t *win, double *out, TypedArgs *ap, bool *empty) {
  if (!dtype_size(dtype)) return fail(BLDP_EINVAL, "unknown element type %d", dtype);
  Geo g;
  int rc = resolve_window(nchan, nif, ntime, win, &g);
  if (rc) return rc;
  TypedArgs &a = *ap;
  a = TypedArgs{};
  a.dtype = dtype;
  a.nbank = 1;
  a.in[0] = in;
  a.out = out;
  a.in_off = g.off;
  a.in_cs = g.cs;
  a.in_ld_i = g.ld_i;
  a.in_ld_t = g.ld_t;
  a.nco = g.nc;
  a.ni = g.ni;
  a.nto = g.nt;
  a.F = a.T = 1;
  a.num_cus = num_cus_current();
  *empty = a.nco * a.ni == 0;
  if (*empty) return BLDP_OK;
  if (!out || (!in && g.nt > 0)) return fail(BLDP_EINVAL, "null pointer");
  return BLDP_OK;
}
}  // namespace

extern "C" {

int bldp_reduce_strided(int dtype, const void *in, int64_t nchan, int64_t nif, int64_t ntime,
                        const int64_t *win, int64_t fqavby, int64_t tavby, int op, void *out,
                        int64_t out_ld_i, int64_t out_ld_t, void *stream) {
  if (dtype == BLDP_DT_F32)
    return bldp_reduce_strided_f32(static_cast<const float *>(in), nchan, nif, ntime, win, fqavby,
                                   tavby, op, static_cast<float *>(out), out_ld_i, out_ld_t,
                                   stream);
  TypedArgs a;
  bool empty = false;
  int rc = typed_reduce_args(dtype, in, nchan, nif, ntime, win, fqavby, tavby, op, out, out_ld_i,
                             out_ld_t, &a, &empty);
  if (rc || empty) return rc;
  hipError_t e = launch_reduce_typed(a, op, (hipStream_t)stream);
  if (e != hipSuccess) return fail(BLDP_EHIP, "typed reduce launch: %s", hipGetErrorString(e));
  return BLDP_OK;
}

int bldp_kurtosis(int dtype, const void *in, int64_t nchan, int64_t nif, int64_t ntime,
                  const int64_t *win, double *out, void *stream) {
  if (dtype == BLDP_DT_F32)
    return bldp_kurtosis_f32(static_cast<const float *>(in), nchan, nif, ntime, win, out, nullptr,
                             stream);
  TypedArgs a;
  bool empty = false;
  int rc = typed_kurt_args(dtype, in, nchan, nif, ntime, win, out, &a, &empty);
  if (rc || empty) return rc;
  ScratchLease lease;  // time-chunk partial sums (k_kurt_i8), held until queued
  if (const size_t wsb = kurtosis_typed_ws_bytes(a)) {
    rc = scratch_lease((hipStream_t)stream, wsb, &lease);
    if (rc) return rc;
    a.ws = lease.ptr;
    a.ws_bytes = wsb;
  }
  hipError_t e = launch_kurtosis_typed(a, out, (hipStream_t)stream);
  if (e != hipSuccess) return fail(BLDP_EHIP, "typed kurtosis launch: %s", hipGetErrorString(e));
  return BLDP_OK;
}

// bldp_reduce_strided / bldp_kurtosis prepared once (any element type): a
// launch through bldp_reduce_launch is one kernel launch (two for the typed
// getkurtosis of long rows), no argument handling.
int bldp_reduce_prepare(int dtype, const void *in, int64_t nchan, int64_t nif, int64_t ntime,
                        const int64_t *win, int64_t fqavby, int64_t tavby, int op, void *out,
                        int64_t out_ld_i, int64_t out_ld_t, bldp_reduce_op_t *handle) {
  if (!handle) return fail(BLDP_EINVAL, "null handle pointer");
  *handle = nullptr;
  auto *h = new (std::nothrow) bldp_reduce_op{};
  if (!h) return fail(BLDP_ENOMEM, "out of host memory");
  int rc;
  if (dtype == BLDP_DT_F32) {
    h->kind = bldp_reduce_op::F32_REDUCE;
    const float *ins[1] = {static_cast<const float *>(in)};
    rc = prepare_reduce(1, ins, nchan, nif, ntime, win, fqavby, tavby, op,
                        static_cast<float *>(out), 0, out_ld_i, out_ld_t, false, false, &h->a,
                        &h->p, &h->empty);
  } else {
    h->kind = bldp_reduce_op::TYPED_REDUCE;
    rc = typed_reduce_args(dtype, in, nchan, nif, ntime, win, fqavby, tavby, op, out, out_ld_i,
                           out_ld_t, &h->t, &h->empty);
  }
  if (rc == BLDP_OK && hipGetDevice(&h->dev) != hipSuccess)
    rc = fail(BLDP_EHIP, "hipGetDevice failed");
  if (rc) {
    delete h;
    return rc;
  }
  h->op = op;
  *handle = h;
  return BLDP_OK;
}

int bldp_kurtosis_prepare(int dtype, const void *in, int64_t nchan, int64_t nif, int64_t ntime,
                          const int64_t *win, double *out, bldp_reduce_op_t *handle) {
  if (!handle) return fail(BLDP_EINVAL, "null handle pointer");
  *handle = nullptr;
  auto *h = new (std::nothrow) bldp_reduce_op{};
  if (!h) return fail(BLDP_ENOMEM, "out of host memory");
  int rc;
  if (dtype == BLDP_DT_F32) {
    h->kind = bldp_reduce_op::F32_KURT;
    const float *ins[1] = {static_cast<const float *>(in)};
    rc = kurt_setup(1, ins, nchan, nif, ntime, win, &h->k);
    h->empty = false;
  } else {
    h->kind = bldp_reduce_op::TYPED_KURT;
    rc = typed_kurt_args(dtype, in, nchan, nif, ntime, win, out, &h->t, &h->empty);
  }
  if (rc == BLDP_OK && hipGetDevice(&h->dev) != hipSuccess)
    rc = fail(BLDP_EHIP, "hipGetDevice failed");
  if (rc) {
    delete h;
    return rc;
  }
  h->kout = out;
  h->op = 0;
  *handle = h;
  return BLDP_OK;
}

int bldp_fqav_range(double first, double step, int64_t len, int64_t n, double *out_first,
                    double *out_step, int64_t *out_len) {
  if (!out_first || !out_step || !out_len) return fail(BLDP_EINVAL, "null pointer");
  if (len < 0) return fail(BLDP_EINVAL, "negative range length");
  if (n <= 1) {  // src/gbtworkerfunctions.jl:28
    *out_first = first;
    *out_step = step;
    *out_len = len;
    return BLDP_OK;
  }
  *out_first = first + (double)(n - 1) * step / 2.0;  // :29
  *out_step = (double)n * step;                        // :30
  *out_len = len / n;                                  // :31 (floor)
  return BLDP_OK;
}

int bldp_unchunk_f32(const float *packed, const int64_t chunk[3], const int64_t box0[3],
                     const int64_t grid[3], const int64_t *win, float *out, void *stream) {
  if (!chunk || !box0 || !grid || !win) return fail(BLDP_EINVAL, "null pointer");
  UnchunkArgs u{chunk[0], chunk[1], chunk[2], box0[0], box0[1], box0[2], grid[0], grid[1],
                grid[2], win[0], win[1], win[2], win[3], win[4], win[5], win[6], win[7], win[8]};
  if (u.ct <= 0 || u.ci <= 0 || u.cc <= 0 || u.gt <= 0 || u.gi <= 0 || u.gc <= 0)
    return fail(BLDP_EINVAL, "bad chunk geometry");
  // every window element must fall inside the chunk box (no out-of-range reads)
  const int64_t ext[3][3] = {{u.c0, u.nc, u.cs}, {u.i0, u.ni, u.is}, {u.t0, u.nt, u.ts}};
  const int64_t lo[3] = {u.bc0, u.bi0, u.bt0}, len[3] = {u.gc * u.cc, u.gi * u.ci, u.gt * u.ct};
  for (int a = 0; a < 3; ++a) {
    if (ext[a][1] < 0) return fail(BLDP_EINVAL, "negative window count");
    if (ext[a][1] == 0) return BLDP_OK;
    // counts and steps beyond the box cannot stay inside it; checked first so
    // the last-index product below cannot overflow
    if (ext[a][1] > 1 && (ext[a][1] > len[a] || ext[a][2] > len[a] || ext[a][2] < -len[a]))
      return fail(BLDP_EBOUNDS, "window axis %d outside the decoded chunk box", a + 1);
    const int64_t first = ext[a][0], last = ext[a][0] + (ext[a][1] - 1) * ext[a][2];
    if (std::min(first, last) < lo[a] || std::max(first, last) >= lo[a] + len[a])
      return fail(BLDP_EBOUNDS, "window axis %d outside the decoded chunk box", a + 1);
  }
  if (!packed || !out) return fail(BLDP_EINVAL, "null pointer");
  hipError_t e = launch_unchunk(packed, u, out, (hipStream_t)stream);
  if (e != hipSuccess) return fail(BLDP_EHIP, "unchunk launch: %s", hipGetErrorString(e));
  return BLDP_OK;
}

int bldp_synth_f32(float *out, int64_t nchan, int64_t nif, int64_t ntime, int64_t nfpc,
                   uint64_t seed, int kind, void *stream) {
  if (nchan < 0 || nif < 0 || ntime < 0) return fail(BLDP_EINVAL, "negative dimension");
  if (kind != 0 && kind != 1) return fail(BLDP_EINVAL, "unknown synth kind %d", kind);
  if (nfpc < 1) return fail(BLDP_EINVAL, "nfpc must be >= 1");
  if (nchan * nif * ntime > 0 && !out) return fail(BLDP_EINVAL, "null pointer");
  hipError_t e = launch_synth(out, nchan, nif, ntime, nfpc, seed, kind, (hipStream_t)stream);
  if (e != hipSuccess) return fail(BLDP_EHIP, "synth launch: %s", hipGetErrorString(e));
  return BLDP_OK;
}

}  // extern "C"
