/*
 * bldp_oracle.c — TEST INFRASTRUCTURE ONLY.  CPU restatement of the
 * reference's worker-side reduction (BLDistributedDataProducts.jl v0.3.2).
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load this library; the product (libbldp_hip) never links or calls it.
 *
 * Parity status: the reference is pure Julia and cannot run here (julia is
 * absent).  Its own tests pin only the range method
 * of fqav (test/runtests.jl:5-6), which oracle_fqav_range reproduces.  The
 * array reductions are PARITY UNPINNED against reference outputs; they are
 * restated line by line below and cross-checked against an independent NumPy
 * restatement (oracle/oracle.py) and against integer-valued fixtures whose
 * sums are exact in any summation order.
 *
 * Numerics: sum/mean accumulate in float64 and round once to float32
 * (Julia's Float32 `sum(...; dims=1)` reassociates under @simd, so its exact
 * bits are machine and version dependent; the GPU path is held to 1e-5
 * relative of this value).  max/min follow Julia's max/min exactly: NaN
 * propagates and -0.0 < +0.0.
 */
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define OP_SUM 0
#define OP_MEAN 1
#define OP_MAX 2
#define OP_MIN 3

/* Julia Base max/min on Float32 (NaN-propagating, -0.0 < +0.0). */
static float jmax(float a, float b) {
  if (a != a) return a;
  if (b != b) return b;
  if (a == b) return signbit(a) ? b : a;
  return a > b ? a : b;
}
static float jmin(float a, float b) {
  if (a != a) return a;
  if (b != b) return b;
  if (a == b) return signbit(a) ? a : b;
  return a < b ? a : b;
}

/* Window resolution: a Julia index tuple (sanitizeidxs, :167-169) becomes,
 * per axis, a 0-based start, a count and a step.  NULL = (:,:,:) (:182-183).
 * Returns 0, -1 (invalid) or -6 (out of bounds). */
typedef struct {
  int64_t nc, ni, nt, off, cs, ldi, ldt;
} geo_t;

static int resolve(int64_t nchan, int64_t nif, int64_t ntime, const int64_t *win, geo_t *g) {
  const int64_t dims[3] = {nchan, nif, ntime};
  int64_t st[3], ct[3], sp[3];
  for (int a = 0; a < 3; ++a) {
    st[a] = win ? win[3 * a] : 0;
    ct[a] = win ? win[3 * a + 1] : dims[a];
    sp[a] = win ? win[3 * a + 2] : 1;
    if (ct[a] < 0) return -1;
    if (ct[a] > 0) {
      int64_t last = st[a] + (ct[a] - 1) * sp[a];
      if (sp[a] == 0) return -1;
      if (st[a] < 0 || st[a] >= dims[a] || last < 0 || last >= dims[a]) return -6;
    }
  }
  g->nc = ct[0];
  g->ni = ct[1];
  g->nt = ct[2];
  g->off = st[0] + nchan * (st[1] + nif * st[2]);
  g->cs = sp[0];
  g->ldi = nchan * sp[1];
  g->ldt = nchan * nif * sp[2];
  return 0;
}

/*
 * fqav(A, n; f) (src/gbtworkerfunctions.jl:16-20) on the channel axis fused
 * with the time integration extension (fqav on axis 3):
 *   out[c', i, t'] = f( A[(c'-1)F+1 : c'F, i, (t'-1)T+1 : t'T] )
 * :17  n <= 1 returns A            -> F (T) <= 1 means "no reduction"
 * :18  reshape(A, (n, :, ...))     -> DimensionMismatch unless n | size(A,1): -2
 * :19  dropdims(f(...; dims=1))    -> one value per group
 * Output dense (nco, ni, nto), Julia column-major.
 */
/* Outputs [co0, co1) of IF row i, time block to (the body of oracle_reduce). */
static void reduce_range(const float *in, const geo_t *g, int64_t F, int64_t T, int op, float *out,
                         int64_t nco, int64_t i, int64_t to, int64_t co0, int64_t co1) {
  for (int64_t co = co0; co < co1; ++co) {
    const float *p = in + g->off + i * g->ldi + to * T * g->ldt + co * F * g->cs;
    float *o = out + co + nco * (i + g->ni * to);
    if (op == OP_SUM || op == OP_MEAN) {
      double acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
      for (int64_t tt = 0; tt < T; ++tt) {
        const float *r = p + tt * g->ldt;
        int64_t k = 0;
        if (g->cs == 1)
          for (; k + 8 <= F; k += 8)
            for (int u = 0; u < 8; ++u) acc[u] += (double)r[k + u];
        for (; k < F; ++k) acc[0] += (double)r[k * g->cs];
      }
      double s = ((acc[0] + acc[1]) + (acc[2] + acc[3])) + ((acc[4] + acc[5]) + (acc[6] + acc[7]));
      /* Julia's reducedim init is zero(Float32) = +0.0, so an all -0.0
       * group sums to +0.0; 0.0 + s reproduces that. */
      if (op == OP_MEAN) s = s / (double)(F * T);
      *o = (float)(0.0 + s);
    } else {
      float m = op == OP_MAX ? -INFINITY : INFINITY;
      for (int64_t tt = 0; tt < T; ++tt)
        for (int64_t k = 0; k < F; ++k) {
          const float v = p[tt * g->ldt + k * g->cs];
          m = op == OP_MAX ? jmax(m, v) : jmin(m, v);
        }
      *o = m;
    }
  }
}

int oracle_reduce(const float *in, int64_t nchan, int64_t nif, int64_t ntime, const int64_t *win,
                  int64_t fqavby, int64_t tavby, int op, float *out) {
  geo_t g;
  int rc = resolve(nchan, nif, ntime, win, &g);
  if (rc) return rc;
  if (op < OP_SUM || op > OP_MIN) return -1;
  const int64_t F = fqavby <= 1 ? 1 : fqavby, T = tavby <= 1 ? 1 : tavby;
  if (g.nc % F || g.nt % T) return -2;
  const int64_t nco = g.nc / F, nto = g.nt / T;
  for (int64_t to = 0; to < nto; ++to)
    for (int64_t i = 0; i < g.ni; ++i) reduce_range(in, &g, F, T, op, out, nco, i, to, 0, nco);
  return 0;
}

/* Julia Base `sum` of a Float32 vector view (mapreduce_impl): pairwise
 * halving above the 1024-element block, sequential below it. */
static float jl_pairwise_sum(const float *p, int64_t stride, int64_t lo, int64_t hi) {
  if (lo == hi) return p[lo * stride];
  if (hi - lo < 1024) {
    float v = p[lo * stride] + p[(lo + 1) * stride];
    for (int64_t k = lo + 2; k <= hi; ++k) v += p[k * stride];
    return v;
  }
  const int64_t mid = lo + ((hi - lo) >> 1);
  return jl_pairwise_sum(p, stride, lo, mid) + jl_pairwise_sum(p, stride, mid + 1, hi);
}

/*
 * getkurtosis (src/gbtworkerfunctions.jl:197-202): data = getdata(fname, idxs)
 * (no fqav, :198); rows = eachrow(reshape(data, nchan*nif, ntime)) (:199-200);
 * StatsBase.kurtosis(v) = kurtosis(v, mean(v)):
 *   m = mean(v)                      Float32 (sum / length)
 *   z = v[i] - m; z2 = z*z           Float32
 *   cm2 += z2; cm4 += z2*z2          Float64 accumulators
 *   cm4 /= n; cm2 /= n; cm4/(cm2*cm2) - 3.0
 * out is (nc, ni) Float64 (:201).
 */
int oracle_kurtosis(const float *in, int64_t nchan, int64_t nif, int64_t ntime,
                    const int64_t *win, double *out) {
  geo_t g;
  int rc = resolve(nchan, nif, ntime, win, &g);
  if (rc) return rc;
  for (int64_t i = 0; i < g.ni; ++i)
    for (int64_t c = 0; c < g.nc; ++c) {
      const float *p = in + g.off + i * g.ldi + c * g.cs;
      const int64_t n = g.nt;
      float m = n > 0 ? jl_pairwise_sum(p, g.ldt, 0, n - 1) / (float)n : NAN;
      double cm2 = 0.0, cm4 = 0.0;
      for (int64_t t = 0; t < n; ++t) {
        const float z = p[t * g.ldt] - m;
        const float z2 = z * z;
        cm2 += (double)z2;
        cm4 += (double)(z2 * z2);
      }
      cm4 /= (double)n;
      cm2 /= (double)n;
      out[c + g.nc * i] = (cm4 / (cm2 * cm2)) - 3.0;
    }
  return 0;
}

/* mean(v) of every (channel, IF) row of the window: StatsBase's m, the
 * Float32 pairwise sum over time / length (Statistics.mean -> sum / n). */
int oracle_mean_f32(const float *in, int64_t nchan, int64_t nif, int64_t ntime,
                    const int64_t *win, float *out) {
  geo_t g;
  int rc = resolve(nchan, nif, ntime, win, &g);
  if (rc) return rc;
  for (int64_t i = 0; i < g.ni; ++i)
    for (int64_t c = 0; c < g.nc; ++c) {
      const float *p = in + g.off + i * g.ldi + c * g.cs;
      out[c + g.nc * i] = g.nt > 0 ? jl_pairwise_sum(p, g.ldt, 0, g.nt - 1) / (float)g.nt : NAN;
    }
  return 0;
}

/* reduce(vcat, banks) along dim 1 (src/gbt.jl:103): banks are (nc, nif, nt)
 * each, output (nbank*nc, nif, nt). */
int oracle_stitch(int nbank, const float *const *banks, int64_t nc, int64_t nif, int64_t nt,
                  float *out) {
  const int64_t wide = nc * nbank;
  for (int64_t t = 0; t < nt; ++t)
    for (int64_t i = 0; i < nif; ++i)
      for (int b = 0; b < nbank; ++b)
        memcpy(out + wide * (i + nif * t) + b * nc, banks[b] + nc * (i + nif * t),
               (size_t)nc * sizeof(float));
  return 0;
}

/* De-spike (src/gbt.jl:101-102,111): spike = nfpc÷2 + 1 (1-based);
 * d[spike:nfpc:end, :, :] .= d[spike-1:nfpc:end, :, :].  A length mismatch of
 * the two strided ranges is a DimensionMismatch (-2); nfpc < 2 makes
 * spike-1 == 0, a BoundsError (-6). */
int oracle_despike(float *d, int64_t nchan, int64_t nif, int64_t nt, int64_t nfpc) {
  if (nfpc < 2) return -6;
  const int64_t s1 = nfpc / 2 + 1; /* 1-based */
  const int64_t nsp = nchan >= s1 ? (nchan - s1) / nfpc + 1 : 0;
  const int64_t nsr = nchan >= s1 - 1 ? (nchan - (s1 - 1)) / nfpc + 1 : 0;
  if (nsp != nsr) return -2;
  for (int64_t r = 0; r < nif * nt; ++r)
    for (int64_t k = 0; k < nsp; ++k) {
      float *row = d + r * nchan;
      row[(s1 - 1) + k * nfpc] = row[(s1 - 2) + k * nfpc];
    }
  return 0;
}

/* fqav(r::AbstractRange, n) (src/gbtworkerfunctions.jl:27-33). */
void oracle_fqav_range(double first, double step, int64_t len, int64_t n, double *of,
                       double *os, int64_t *ol) {
  if (n <= 1) { /* :28 */
    *of = first;
    *os = step;
    *ol = len;
    return;
  }
  *of = first + (double)(n - 1) * step / 2; /* :29 */
  *os = (double)n * step;                   /* :30 */
  *ol = len / n;                            /* :31 */
}

/* Same generator as the device's bldp_synth_f32 (kind 1 is bit-identical;
 * kind 0 uses libm logf/sinf, so it matches the GPU only to ~1 ulp). */
static uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}
void oracle_synth(float *out, int64_t nchan, int64_t nif, int64_t ntime, int64_t nfpc,
                  uint64_t seed, int kind) {
  const int64_t n = nchan * nif * ntime;
  for (int64_t e = 0; e < n; ++e) {
    const uint64_t h = splitmix64((uint64_t)e + seed * 0xD1B54A32D192ED03ull);
    if (kind == 1) {
      out[e] = (float)(h >> 56);
      continue;
    }
    const float u1 = (float)((h >> 41) + 1) * (1.0f / 8388608.0f);
    const float u2 = (float)(((h >> 17) & 0x7FFFFF) + 1) * (1.0f / 8388608.0f);
    const float gam = -(logf(u1) + logf(u2)) * 5.0e8f;
    const int64_t x = (e % nchan) % nfpc;
    const float s = sinf(3.14159265f * ((float)x + 0.5f) / (float)nfpc);
    float bp = 0.2f + 0.8f * s * s;
    if (x == nfpc / 2) bp *= 10.0f;
    out[e] = gam * bp;
  }
}

/* CPU baseline: one thread per bank, the way GBT.getdata runs one
 * Distributed worker per bank file (src/gbt.jl:75-77).  With nthreads > 0
 * the banks' output channels are instead split into pieces taken by
 * nthreads threads (all cores on one node, same arithmetic). */
typedef struct {
  const float *const *in;
  float *const *out;
  int64_t nchan, nif, ntime, F, T;
  int op, nbank;
  int64_t piece, npiece;        /* outputs per piece, pieces per (bank, i, to) row */
  int64_t next, total;          /* work counter (pieces over every bank and row) */
  pthread_mutex_t mu;
  int rc;
} pool_t;
static void *pool_run(void *arg) {
  pool_t *P = (pool_t *)arg;
  geo_t g;
  resolve(P->nchan, P->nif, P->ntime, NULL, &g);
  const int64_t nco = g.nc / P->F, nto = g.nt / P->T;
  for (;;) {
    pthread_mutex_lock(&P->mu);
    const int64_t w = P->next++;
    pthread_mutex_unlock(&P->mu);
    if (w >= P->total) break;
    const int64_t pc = w % P->npiece, row = w / P->npiece;
    const int64_t b = row / (g.ni * nto), r2 = row % (g.ni * nto), i = r2 % g.ni, to = r2 / g.ni;
    const int64_t co0 = pc * P->piece, co1 = co0 + P->piece < nco ? co0 + P->piece : nco;
    reduce_range(P->in[b], &g, P->F, P->T, P->op, P->out[b], nco, i, to, co0, co1);
  }
  return NULL;
}
int oracle_reduce_banks_pool(int nbank, const float *const *in, int64_t nchan, int64_t nif,
                             int64_t ntime, int64_t F, int64_t T, int op, float *const *out,
                             int nthreads) {
  if (nbank < 1 || nthreads < 1 || nthreads > 1024) return -1;
  const int64_t Fx = F <= 1 ? 1 : F, Tx = T <= 1 ? 1 : T;
  if (nchan % Fx || ntime % Tx) return -2;
  pool_t P;
  P.in = in; P.out = out; P.nchan = nchan; P.nif = nif; P.ntime = ntime; P.F = Fx; P.T = Tx;
  P.op = op; P.nbank = nbank; P.rc = 0; P.next = 0;
  const int64_t nco = nchan / Fx;
  P.piece = nco / 64 > 1 ? nco / 64 : 1;  /* 64 pieces per row */
  P.npiece = (nco + P.piece - 1) / P.piece;
  P.total = P.npiece * nbank * nif * (ntime / Tx);
  pthread_mutex_init(&P.mu, NULL);
  pthread_t th[1024];
  int started = 0;
  for (int t = 0; t < nthreads; ++t)
    if (pthread_create(&th[t], NULL, pool_run, &P) == 0) ++started;
  for (int t = 0; t < started; ++t) pthread_join(th[t], NULL);
  pthread_mutex_destroy(&P.mu);
  return started ? 0 : -1;
}

typedef struct {
  const float *in;
  float *out;
  int64_t nchan, nif, ntime, F, T;
  int op, rc;
} job_t;
static void *run_job(void *p) {
  job_t *j = (job_t *)p;
  j->rc = oracle_reduce(j->in, j->nchan, j->nif, j->ntime, NULL, j->F, j->T, j->op, j->out);
  return NULL;
}
int oracle_reduce_banks_mt(int nbank, const float *const *in, int64_t nchan, int64_t nif,
                           int64_t ntime, int64_t F, int64_t T, int op, float *const *out) {
  pthread_t th[64];
  job_t jobs[64];
  if (nbank < 1 || nbank > 64) return -1;
  for (int b = 0; b < nbank; ++b) {
    jobs[b] = (job_t){in[b], out[b], nchan, nif, ntime, F, T, op, 0};
    if (pthread_create(&th[b], NULL, run_job, &jobs[b])) return -1;
  }
  int rc = 0;
  for (int b = 0; b < nbank; ++b) {
    pthread_join(th[b], NULL);
    if (jobs[b].rc) rc = jobs[b].rc;
  }
  return rc;
}
