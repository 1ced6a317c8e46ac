// host.hip — bldp_reduce_host_f32: the drop-in for a worker that already holds
// the window in host memory (after h5["data"][idxs...] at
// src/gbtworkerfunctions.jl:185 or dmmap[idxs...] at :174).  The window is
// streamed to the GPU in chunks of whole output time rows on the two streams
// of a pooled staging pipeline (runtime.hip; copy of chunk k+1 overlaps the
// reduce of chunk k) and the reduced rows come back into the caller's dense
// (nco, ni, nto) buffer.  Nothing is allocated per call.
#include <math.h>

#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <string>

#include "bldp_impl.h"

extern "C" int bldp_reduce_shape(int64_t, int64_t, int64_t, const int64_t *, int64_t, int64_t,
                                 int64_t *);
extern "C" int bldp_kurtosis_f32(const float *, int64_t, int64_t, int64_t, const int64_t *,
                                 double *, void *, void *);
extern "C" int bldp_reduce_strided_f32(const float *, int64_t, int64_t, int64_t,
                                       const int64_t *, int64_t, int64_t, int, float *, int64_t,
                                       int64_t, void *);
extern "C" int bldp_reduce_strided(int, const void *, int64_t, int64_t, int64_t, const int64_t *,
                                   int64_t, int64_t, int, void *, int64_t, int64_t, void *);
extern "C" int bldp_kurtosis(int, const void *, int64_t, int64_t, int64_t, const int64_t *,
                             double *, void *);
extern "C" int bldp_reduce_out_dtype(int, int);

namespace {

struct DevGuard {
  int prev = -1;
  explicit DevGuard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    (void)hipSetDevice(dev);
  }
  ~DevGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};

#define HCHK(x)                                                             \
  do {                                                                      \
    hipError_t e_ = (x);                                                    \
    if (e_ != hipSuccess)                                                   \
      return bldp::set_error(BLDP_EHIP, "%s: %s", #x, hipGetErrorString(e_)); \
  } while (0)

// Run `body` on an idle staging pipeline of `dev`; both of its streams are
// drained before the pipeline goes back to the pool (also after an error), so
// no copy into caller memory is pending when the entry point returns.
template <class Body>
int with_stager(int dev, Body body) {
  bldp::Stager *sg = nullptr;
  int rc = bldp::stager_acquire(dev, &sg);
  if (rc) return rc;
  {
    DevGuard guard(dev);
    rc = body(sg);
    for (int b = 0; b < 2; ++b) {
      const hipError_t e = hipStreamSynchronize(sg->st[b]);
      if (e != hipSuccess && rc == BLDP_OK)
        rc = bldp::set_error(BLDP_EHIP, "device %d: %s", dev, hipGetErrorString(e));
    }
  }
  bldp::stager_release(sg);
  return rc;
}

// Staged window rows: element (c, i, t) of the window at
// row0[c*cs' + i*ld_i + t*ld_t] (elements of esz bytes) with c counted from the
// lowest channel touched.
struct HostWin {
  int64_t nc, cs, acs, span, ni, ld_i, ld_t, esz;
  const char *row0;
  bool uniform;   // rows are a single 2-D copy
  int64_t pitch;  // of that copy, in elements
};

HostWin host_window(const void *in, int64_t esz, int64_t nchan, int64_t nif, const int64_t *win,
                    int64_t nc, int64_t ni) {
  HostWin h;
  h.esz = esz;
  const int64_t c0 = win ? win[0] : 0, cs = win ? win[2] : 1;
  const int64_t i0 = win ? win[3] : 0, is = win ? win[5] : 1;
  const int64_t t0 = win ? win[6] : 0, ts = win ? win[8] : 1;
  h.nc = nc;
  h.ni = ni;
  h.cs = cs;
  h.acs = cs < 0 ? -cs : cs;
  h.span = (nc - 1) * h.acs + 1;                        // staged floats per (i, t) row
  const int64_t c_lo = cs < 0 ? c0 + (nc - 1) * cs : c0;  // lowest channel touched
  h.ld_i = nchan * is;
  h.ld_t = nchan * nif * ts;
  h.row0 = static_cast<const char *>(in) + (c_lo + nchan * (i0 + nif * t0)) * esz;
  h.uniform = (ni == 1 && h.ld_t > 0 && h.ld_t >= h.span) ||
              (h.ld_i > 0 && h.ld_i >= h.span && h.ld_t == ni * h.ld_i);
  h.pitch = ni == 1 ? h.ld_t : h.ld_i;
  return h;
}

// Copy `rows` window time rows starting at window row r0 into dense
// [t][i][span] device memory.
int stage_rows(const HostWin &h, int64_t r0, int64_t rows, void *dstv, hipStream_t st) {
  const int64_t e = h.esz;
  const char *src = h.row0 + r0 * h.ld_t * e;
  char *dst = static_cast<char *>(dstv);
  if (h.uniform) {
    HCHK(hipMemcpy2DAsync(dst, h.span * e, src, h.pitch * e, h.span * e, (size_t)(rows * h.ni),
                          hipMemcpyHostToDevice, st));
  } else {
    for (int64_t r = 0; r < rows; ++r)
      for (int64_t i = 0; i < h.ni; ++i)
        HCHK(hipMemcpyAsync(dst + (r * h.ni + i) * h.span * e, src + (r * h.ld_t + i * h.ld_i) * e,
                            h.span * e, hipMemcpyHostToDevice, st));
  }
  return BLDP_OK;
}

}  // namespace

extern "C" int bldp_reduce_host_f32(int dev, const float *in, int64_t nchan, int64_t nif,
                                    int64_t ntime, const int64_t *win, int64_t fqavby,
                                    int64_t tavby, int op, float *out) {
  int64_t sh[3];
  int rc = bldp_reduce_shape(nchan, nif, ntime, win, fqavby, tavby, sh);
  if (rc) return rc;
  const int64_t nco = sh[0], ni = sh[1], nto = sh[2];
  if (nco * ni * nto == 0) return BLDP_OK;
  if (!in || !out) return bldp::set_error(BLDP_EINVAL, "null pointer");
  const int64_t F = fqavby <= 1 ? 1 : fqavby, T = tavby <= 1 ? 1 : tavby;
  const HostWin h = host_window(in, 4, nchan, nif, win, nco * F, ni);

  // chunk = q output time rows (q*T input rows), ~128 MiB of staged input
  const int64_t row_bytes = h.span * ni * (int64_t)sizeof(float);
  int64_t q = std::max<int64_t>(1, ((int64_t)128 << 20) / std::max<int64_t>(1, row_bytes * T));
  q = std::min(q, nto);
  const int64_t nchunks = (nto + q - 1) / q;
  return with_stager(dev, [&](bldp::Stager *sg) -> int {
    float *dbuf[2], *dout[2];
    for (int b = 0; b < 2 && b < nchunks; ++b) {
      int r = bldp::stager_buffer(sg, b, (size_t)(q * T) * row_bytes, (void **)&dbuf[b]);
      if (!r) r = bldp::stager_buffer(sg, 2 + b, (size_t)(nco * ni * q) * sizeof(float),
                                     (void **)&dout[b]);
      if (r) return r;
    }
    for (int64_t k = 0; k < nchunks; ++k) {
      const int b = (int)(k & 1);
      const int64_t to0 = k * q, qn = std::min(q, nto - to0), rows = qn * T;
      int r = stage_rows(h, to0 * T, rows, dbuf[b], sg->st[b]);
      if (r) return r;
      const int64_t dwin[9] = {h.cs < 0 ? (h.nc - 1) * h.acs : 0, h.nc, h.cs, 0, ni, 1, 0, rows, 1};
      r = bldp_reduce_strided_f32(dbuf[b], h.span, ni, rows, dwin, F, T, op, dout[b], nco,
                                  nco * ni, sg->st[b]);
      if (r) return r;  // message already recorded
      HCHK(hipMemcpyAsync(out + to0 * nco * ni, dout[b], (size_t)(nco * ni * qn) * sizeof(float),
                          hipMemcpyDeviceToHost, sg->st[b]));
    }
    return BLDP_OK;
  });
}

// Stage the window rows ([t][i][span] dense) on the device with the same copy
// rules as bldp_reduce_host_f32, then run the two-pass kurtosis there.
extern "C" int bldp_kurtosis_host_f32(int dev, const float *in, int64_t nchan, int64_t nif,
                                      int64_t ntime, const int64_t *win, double *out) {
  int64_t sh[3];
  int rc = bldp_reduce_shape(nchan, nif, ntime, win, 1, 1, sh);
  if (rc) return rc;
  const int64_t nc = sh[0], ni = sh[1], nt = sh[2];
  if (nc * ni == 0) return BLDP_OK;
  if (!out || (!in && nt > 0)) return bldp::set_error(BLDP_EINVAL, "null pointer");
  const HostWin h = host_window(in, 4, nchan, nif, win, nc, ni);
  return with_stager(dev, [&](bldp::Stager *sg) -> int {
    float *dbuf;
    double *dout;
    int r = bldp::stager_buffer(sg, 0, (size_t)std::max<int64_t>(1, h.span * ni * nt) * 4,
                                (void **)&dbuf);
    if (!r) r = bldp::stager_buffer(sg, 2, (size_t)(nc * ni) * sizeof(double), (void **)&dout);
    if (!r && nt > 0) r = stage_rows(h, 0, nt, dbuf, sg->st[0]);
    if (r) return r;
    const int64_t dwin[9] = {h.cs < 0 ? (nc - 1) * h.acs : 0, nc, h.cs, 0, ni, 1, 0, nt, 1};
    r = bldp_kurtosis_f32(dbuf, h.span, ni, nt, dwin, dout, nullptr, sg->st[0]);
    if (r) return r;
    HCHK(hipMemcpyAsync(out, dout, (size_t)(nc * ni) * sizeof(double), hipMemcpyDeviceToHost,
                        sg->st[0]));
    return BLDP_OK;
  });
}

// ---------------------------------------------------------------------------
// Host forms of the typed entry points (include/bldp.h), staged like the
// Float32 forms above: only the window's rows (its channel span of every
// selected (IF, spectrum) row) cross to the device, dense [t][i][span], so a
// narrow window of a large mmap'ed SIGPROC file moves the window, not the file.
// The reduce runs in chunks of whole output time rows on the two streams of a
// pooled staging pipeline; the kurtosis, which needs every spectrum of a row,
// stages the window once.  Synchronous.
extern "C" int bldp_reduce_host(int dev, int dtype, const void *in, int64_t nchan, int64_t nif,
                                int64_t ntime, const int64_t *win, int64_t fqavby, int64_t tavby,
                                int op, void *out) {
  if (dtype == BLDP_DT_F32)
    return bldp_reduce_host_f32(dev, static_cast<const float *>(in), nchan, nif, ntime, win,
                                fqavby, tavby, op, static_cast<float *>(out));
  const int od = bldp_reduce_out_dtype(dtype, op);
  if (od < 0) return od;
  int64_t sh[3];
  int rc = bldp_reduce_shape(nchan, nif, ntime, win, fqavby, tavby, sh);
  if (rc) return rc;
  const int64_t nco = sh[0], ni = sh[1], nto = sh[2];
  if (nco * ni * nto == 0) return BLDP_OK;
  if (!in || !out) return bldp::set_error(BLDP_EINVAL, "null pointer");
  const int64_t esz = (int64_t)bldp::dtype_size(dtype), osz = (int64_t)bldp::dtype_size(od);
  const int64_t F = fqavby <= 1 ? 1 : fqavby, T = tavby <= 1 ? 1 : tavby;
  const HostWin h = host_window(in, esz, nchan, nif, win, nco * F, ni);
  const int64_t row_bytes = h.span * ni * esz;
  int64_t q = std::max<int64_t>(1, ((int64_t)128 << 20) / std::max<int64_t>(1, row_bytes * T));
  q = std::min(q, nto);
  const int64_t nchunks = (nto + q - 1) / q;
  return with_stager(dev, [&](bldp::Stager *sg) -> int {
    void *dbuf[2], *dout[2];
    for (int b = 0; b < 2 && b < nchunks; ++b) {
      int r = bldp::stager_buffer(sg, b, (size_t)(q * T * row_bytes), &dbuf[b]);
      if (!r) r = bldp::stager_buffer(sg, 2 + b, (size_t)(nco * ni * q * osz), &dout[b]);
      if (r) return r;
    }
    for (int64_t k = 0; k < nchunks; ++k) {
      const int b = (int)(k & 1);
      const int64_t to0 = k * q, qn = std::min(q, nto - to0), rows = qn * T;
      int r = stage_rows(h, to0 * T, rows, dbuf[b], sg->st[b]);
      if (r) return r;
      const int64_t dwin[9] = {h.cs < 0 ? (h.nc - 1) * h.acs : 0, h.nc, h.cs, 0, ni, 1, 0, rows, 1};
      r = bldp_reduce_strided(dtype, dbuf[b], h.span, ni, rows, dwin, F, T, op, dout[b], nco,
                              nco * ni, sg->st[b]);
      if (r) return r;
      HCHK(hipMemcpyAsync(static_cast<char *>(out) + to0 * nco * ni * osz, dout[b],
                          (size_t)(nco * ni * qn * osz), hipMemcpyDeviceToHost, sg->st[b]));
    }
    return BLDP_OK;
  });
}

extern "C" int bldp_kurtosis_host(int dev, int dtype, const void *in, int64_t nchan, int64_t nif,
                                  int64_t ntime, const int64_t *win, double *out) {
  if (dtype == BLDP_DT_F32)
    return bldp_kurtosis_host_f32(dev, static_cast<const float *>(in), nchan, nif, ntime, win,
                                  out);
  if (!bldp::dtype_size(dtype)) return bldp::set_error(BLDP_EINVAL, "unknown element type %d", dtype);
  int64_t sh[3];
  int rc = bldp_reduce_shape(nchan, nif, ntime, win, 1, 1, sh);
  if (rc) return rc;
  const int64_t nc = sh[0], ni = sh[1], nt = sh[2];
  if (nc * ni == 0) return BLDP_OK;
  if (!out) return bldp::set_error(BLDP_EINVAL, "null pointer");
  if (nt == 0) {  // no spectra: every row NaN (mean of nothing), as the Float32 path
    for (int64_t k = 0; k < nc * ni; ++k) out[k] = NAN;
    return BLDP_OK;
  }
  if (!in) return bldp::set_error(BLDP_EINVAL, "null pointer");
  const int64_t esz = (int64_t)bldp::dtype_size(dtype);
  const HostWin h = host_window(in, esz, nchan, nif, win, nc, ni);
  return with_stager(dev, [&](bldp::Stager *sg) -> int {
    void *dbuf, *dout;
    int r = bldp::stager_buffer(sg, 0, (size_t)(h.span * ni * nt * esz), &dbuf);
    if (!r) r = bldp::stager_buffer(sg, 2, (size_t)(nc * ni) * sizeof(double), &dout);
    if (!r) r = stage_rows(h, 0, nt, dbuf, sg->st[0]);
    if (r) return r;
    const int64_t dwin[9] = {h.cs < 0 ? (nc - 1) * h.acs : 0, nc, h.cs, 0, ni, 1, 0, nt, 1};
    r = bldp_kurtosis(dtype, dbuf, h.span, ni, nt, dwin, static_cast<double *>(dout), sg->st[0]);
    if (r) return r;
    HCHK(hipMemcpyAsync(out, dout, (size_t)(nc * ni) * sizeof(double), hipMemcpyDeviceToHost,
                        sg->st[0]));
    return BLDP_OK;
  });
}
