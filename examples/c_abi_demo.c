/*
 * c_abi_demo.c — libbldp_hip driven from plain C, the way the Julia
 * reference's worker would drive it through ccall: host
 * arrays in Julia's (nchan, nif, ntime) column-major layout, a 9-int window
 * for idxs, int return codes plus bldp_last_error.  No HIP or torch here.
 *
 *   gcc -O2 -std=c11 examples/c_abi_demo.c -Iinclude \
 *       -Lbldistributeddataproducts.jl_amd -lbldp_hip -lm -o build/c_abi_demo
 *
 * Runs on a GPU box; exits 0 when every check passes.
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "bldp.h"

static int fails = 0;
#define CHECK(cond, ...)                     \
  do {                                       \
    if (!(cond)) {                           \
      fprintf(stderr, "FAIL: " __VA_ARGS__); \
      fprintf(stderr, "\n");                 \
      ++fails;                               \
    }                                        \
  } while (0)

static uint64_t lcg = 12345;
static float next_int255(void) {
  lcg = lcg * 6364136223846793005ull + 1442695040888963407ull;
  return (float)((lcg >> 33) % 256);
}

int main(void) {
  /* a 0002-shaped bank: 65536 channels x 1 IF x 279 spectra, Julia order */
  const int64_t nchan = 65536, nif = 1, ntime = 279;
  const size_t n = (size_t)(nchan * nif * ntime);
  float *a = malloc(n * sizeof(float));
  for (size_t k = 0; k < n; ++k) a[k] = next_int255(); /* integers: exact sums */

  int rc = bldp_init(0, NULL);
  CHECK(rc == BLDP_OK, "bldp_init rc=%d", rc);

  /* getdata(f, (:, :, 1:272); fqavby=64, tavby=16) */
  const int64_t win[9] = {0, nchan, 1, 0, nif, 1, 0, 272, 1};
  int64_t shp[3];
  rc = bldp_reduce_shape(nchan, nif, ntime, win, 64, 16, shp);
  CHECK(rc == BLDP_OK && shp[0] == 1024 && shp[1] == 1 && shp[2] == 17, "reduce_shape");
  float *out = malloc((size_t)(shp[0] * shp[1] * shp[2]) * sizeof(float));
  rc = bldp_reduce_host_f32(0, a, nchan, nif, ntime, win, 64, 16, BLDP_OP_SUM, out);
  CHECK(rc == BLDP_OK, "reduce_host rc=%d", rc);
  int bad = 0;
  for (int64_t to = 0; to < shp[2]; ++to)
    for (int64_t co = 0; co < shp[0]; ++co) {
      double s = 0;
      for (int64_t t = to * 16; t < to * 16 + 16; ++t)
        for (int64_t c = co * 64; c < co * 64 + 64; ++c) s += a[t * nchan + c];
      if ((float)s != out[to * shp[0] + co]) ++bad;
    }
  CHECK(bad == 0, "%d of %lld reduced values differ", bad, (long long)(shp[0] * shp[2]));

  /* max over fqavby=8 of channels 1025:2048 (a misaligned window) */
  const int64_t w2[9] = {1024, 1024, 1, 0, 1, 1, 0, ntime, 1};
  float *mx = malloc(128 * ntime * sizeof(float));
  rc = bldp_reduce_host_f32(0, a, nchan, nif, ntime, w2, 8, 1, BLDP_OP_MAX, mx);
  CHECK(rc == BLDP_OK, "reduce_host max rc=%d", rc);
  bad = 0;
  for (int64_t t = 0; t < ntime; ++t)
    for (int64_t co = 0; co < 128; ++co) {
      float m = -INFINITY;
      for (int64_t c = 1024 + co * 8; c < 1024 + co * 8 + 8; ++c)
        m = a[t * nchan + c] > m ? a[t * nchan + c] : m;
      if (m != mx[t * 128 + co]) ++bad;
    }
  CHECK(bad == 0, "%d max values differ", bad);

  /* getkurtosis(f, (1:256, :, :)): StatsBase recipe, Float64 out */
  const int64_t w3[9] = {0, 256, 1, 0, 1, 1, 0, ntime, 1};
  double *ku = malloc(256 * sizeof(double));
  rc = bldp_kurtosis_host_f32(0, a, nchan, nif, ntime, w3, ku);
  CHECK(rc == BLDP_OK, "kurtosis_host rc=%d", rc);
  bad = 0;
  for (int64_t c = 0; c < 256; ++c) {
    double s = 0;
    for (int64_t t = 0; t < ntime; ++t) s += a[t * nchan + c];
    const float m = (float)s / (float)ntime;
    double c2 = 0, c4 = 0;
    for (int64_t t = 0; t < ntime; ++t) {
      const float z = a[t * nchan + c] - m, z2 = z * z;
      c2 += z2;
      c4 += (double)(z2 * z2);
    }
    c2 /= ntime;
    c4 /= ntime;
    const double k = c4 / (c2 * c2) - 3.0;
    if (fabs(ku[c] - k) > 1e-4 * fabs(k) + 1e-5) ++bad;
  }
  CHECK(bad == 0, "%d kurtosis values differ", bad);

  /* fqav(1:2:15, 4) === 4.0:8.0:12.0 (test/runtests.jl:6) */
  double f0, st;
  int64_t len;
  rc = bldp_fqav_range(1.0, 2.0, 8, 4, &f0, &st, &len);
  CHECK(rc == BLDP_OK && f0 == 4.0 && st == 8.0 && len == 2, "fqav_range");

  /* errors: DimensionMismatch and BoundsError, with a message */
  rc = bldp_reduce_host_f32(0, a, nchan, nif, ntime, win, 3, 1, BLDP_OP_SUM, out);
  char msg[256];
  bldp_last_error(msg, sizeof msg);
  CHECK(rc == BLDP_EDIM && strstr(msg, "DimensionMismatch"), "EDIM: rc=%d msg=%s", rc, msg);
  const int64_t w4[9] = {0, nchan + 1, 1, 0, 1, 1, 0, 16, 1};
  rc = bldp_reduce_host_f32(0, a, nchan, nif, ntime, w4, 1, 1, BLDP_OP_SUM, out);
  CHECK(rc == BLDP_EBOUNDS, "EBOUNDS: rc=%d", rc);

  rc = bldp_finalize();
  CHECK(rc == BLDP_OK, "bldp_finalize rc=%d", rc);
  free(a);
  free(out);
  free(mx);
  free(ku);
  if (fails) return 1;
  printf("c_abi_demo: all checks passed\n");
  return 0;
}
