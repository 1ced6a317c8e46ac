// host.hip — bldp_reduce_host_f32: the drop-in for a worker that already holds
// the window in host memory (after h5["data"][idxs...] at
// src/gbtworkerfunctions.jl:185 or dmmap[idxs...] at :174).  The window is
// streamed to the GPU in chunks of whole output time rows on two HIP streams
// (copy of chunk k+1 overlaps the reduce of chunk k) and the reduced rows come
// back into the caller's dense (nco, ni, nto) buffer.
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

}  // namespace

#define HCHK(x)                                                         \
  do {                                                                  \
    hipError_t e_ = (x);                                                \
    if (e_ != hipSuccess) {                                             \
      rc = bldp::set_error(BLDP_EHIP, "%s: %s", #x, hipGetErrorString(e_)); \
      goto done;                                                        \
    }                                                                   \
  } while (0)

extern "C" int bldp_reduce_host_f32(int dev, const float *in, int64_t nchan, int64_t nif,
                                    int64_t ntime, const int64_t *win, int64_t fqavby,
                                    int64_t tavby, int op, float *out) {
  int64_t sh[3];
  int rc = bldp_reduce_shape(nchan, nif, ntime, win, fqavby, tavby, sh);
  if (rc) return rc;
  const int64_t nco = sh[0], ni = sh[1], nto = sh[2];
  if (nco * ni * nto == 0) return BLDP_OK;
  if (!in || !out) return bldp::set_error(BLDP_EINVAL, "null pointer");
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || dev < 0 || dev >= ndev)
    return bldp::set_error(BLDP_EINVAL, "device %d not available", dev);
  DevGuard guard(dev);

  // window (same conventions as the device path)
  const int64_t c0 = win ? win[0] : 0, nc = win ? win[1] : nchan, cs = win ? win[2] : 1;
  const int64_t i0 = win ? win[3] : 0, is = win ? win[5] : 1;
  const int64_t t0 = win ? win[6] : 0, ts = win ? win[8] : 1;
  const int64_t F = fqavby <= 1 ? 1 : fqavby, T = tavby <= 1 ? 1 : tavby;
  const int64_t acs = cs < 0 ? -cs : cs;
  const int64_t span = (nc - 1) * acs + 1;               // staged floats per (i, t) row
  const int64_t c_lo = cs < 0 ? c0 + (nc - 1) * cs : c0;  // lowest channel touched
  const int64_t ld_i = nchan * is, ld_t = nchan * nif * ts;
  const float *row0 = in + c_lo + nchan * (i0 + nif * t0);

  // chunk = q output time rows (q*T input rows), ~128 MiB of staged input
  const int64_t row_bytes = span * ni * (int64_t)sizeof(float);
  int64_t q = std::max<int64_t>(1, ((int64_t)128 << 20) / std::max<int64_t>(1, row_bytes * T));
  q = std::min(q, nto);
  const int64_t nchunks = (nto + q - 1) / q;
  const bool uniform = (ni == 1 && ld_t > 0 && ld_t >= span) ||
                       (ld_i > 0 && ld_i >= span && ld_t == ni * ld_i);
  const int64_t pitch = ni == 1 ? ld_t : ld_i;

  float *dbuf[2] = {nullptr, nullptr}, *dout[2] = {nullptr, nullptr};
  hipStream_t st[2] = {nullptr, nullptr};
  for (int b = 0; b < 2; ++b) {
    HCHK(hipStreamCreateWithFlags(&st[b], hipStreamNonBlocking));
    HCHK(hipMalloc(&dbuf[b], (size_t)(q * T) * row_bytes));
    HCHK(hipMalloc(&dout[b], (size_t)(nco * ni * q) * sizeof(float)));
  }
  for (int64_t k = 0; k < nchunks; ++k) {
    const int b = (int)(k & 1);
    const int64_t to0 = k * q, qn = std::min(q, nto - to0), rows = qn * T;
    const float *src = row0 + (to0 * T) * ld_t;
    if (uniform) {
      HCHK(hipMemcpy2DAsync(dbuf[b], span * sizeof(float), src, pitch * sizeof(float),
                            span * sizeof(float), (size_t)(rows * ni), hipMemcpyHostToDevice,
                            st[b]));
    } else {
      for (int64_t r = 0; r < rows; ++r)
        for (int64_t i = 0; i < ni; ++i)
          HCHK(hipMemcpyAsync(dbuf[b] + (r * ni + i) * span, src + r * ld_t + i * ld_i,
                              span * sizeof(float), hipMemcpyHostToDevice, st[b]));
    }
    const int64_t dwin[9] = {cs < 0 ? (nc - 1) * acs : 0, nc, cs, 0, ni, 1, 0, rows, 1};
    rc = bldp_reduce_strided_f32(dbuf[b], span, ni, rows, dwin, F, T, op, dout[b], nco,
                                 nco * ni, st[b]);
    if (rc) goto done;  // message already recorded
    HCHK(hipMemcpyAsync(out + to0 * nco * ni, dout[b], (size_t)(nco * ni * qn) * sizeof(float),
                        hipMemcpyDeviceToHost, st[b]));
  }
  for (int b = 0; b < 2; ++b) HCHK(hipStreamSynchronize(st[b]));
done:
  for (int b = 0; b < 2; ++b) {
    if (st[b]) (void)hipStreamSynchronize(st[b]);
    if (dbuf[b]) (void)hipFree(dbuf[b]);
    if (dout[b]) (void)hipFree(dout[b]);
    if (st[b]) (void)hipStreamDestroy(st[b]);
  }
  return rc;
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
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || dev < 0 || dev >= ndev)
    return bldp::set_error(BLDP_EINVAL, "device %d not available", dev);
  DevGuard guard(dev);
  const int64_t c0 = win ? win[0] : 0, cs = win ? win[2] : 1;
  const int64_t i0 = win ? win[3] : 0, is = win ? win[5] : 1;
  const int64_t t0 = win ? win[6] : 0, ts = win ? win[8] : 1;
  const int64_t acs = cs < 0 ? -cs : cs;
  const int64_t span = (nc - 1) * acs + 1;
  const int64_t c_lo = cs < 0 ? c0 + (nc - 1) * cs : c0;
  const int64_t ld_i = nchan * is, ld_t = nchan * nif * ts;
  const float *row0 = in + c_lo + nchan * (i0 + nif * t0);
  float *dbuf = nullptr;
  double *dout = nullptr;
  hipStream_t st = nullptr;
  const int64_t dwin[9] = {cs < 0 ? (nc - 1) * acs : 0, nc, cs, 0, ni, 1, 0, nt, 1};
  HCHK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  HCHK(hipMalloc(&dbuf, (size_t)std::max<int64_t>(1, span * ni * nt) * sizeof(float)));
  HCHK(hipMalloc(&dout, (size_t)(nc * ni) * sizeof(double)));
  if (nt > 0) {
    const bool uniform = (ni == 1 && ld_t > 0 && ld_t >= span) ||
                         (ld_i > 0 && ld_i >= span && ld_t == ni * ld_i);
    if (uniform) {
      const int64_t pitch = ni == 1 ? ld_t : ld_i;
      HCHK(hipMemcpy2DAsync(dbuf, span * sizeof(float), row0, pitch * sizeof(float),
                            span * sizeof(float), (size_t)(nt * ni), hipMemcpyHostToDevice, st));
    } else {
      for (int64_t r = 0; r < nt; ++r)
        for (int64_t i = 0; i < ni; ++i)
          HCHK(hipMemcpyAsync(dbuf + (r * ni + i) * span, row0 + r * ld_t + i * ld_i,
                              span * sizeof(float), hipMemcpyHostToDevice, st));
    }
  }
  rc = bldp_kurtosis_f32(dbuf, span, ni, nt, dwin, dout, nullptr, st);
  if (rc) goto done;
  HCHK(hipMemcpyAsync(out, dout, (size_t)(nc * ni) * sizeof(double), hipMemcpyDeviceToHost, st));
  HCHK(hipStreamSynchronize(st));
done:
  if (st) (void)hipStreamSynchronize(st);
  if (dbuf) (void)hipFree(dbuf);
  if (dout) (void)hipFree(dout);
  if (st) (void)hipStreamDestroy(st);
  return rc;
}
