// kurtosis.hip — getkurtosis (src/gbtworkerfunctions.jl:197-202) on gfx950.
//
// The reference maps StatsBase.kurtosis over the rows of
// reshape(data, nchan*nif, ntime) (:199-200), i.e. over time for every
// (channel, IF):
//   kurtosis(v) = kurtosis(v, mean(v))
//   m    = mean(v)             Float32: Base.sum(v) / length(v)
//   z    = v[i] - m            Float32
//   z2   = z * z               Float32
//   cm2 += z2; cm4 += z2 * z2  Float64 accumulators
//   (cm4 / n) / (cm2 / n)^2 - 3.0
// Base.sum of a Float32 vector (Base.mapreduce_impl, pairwise_blocksize 1024)
// splits the index range in halves (left half ceil(len/2)) until a piece
// holds <= 1024 elements, sums every piece sequentially from its first
// element, and adds the halves back up the tree in Float32.  Every path here
// reproduces that Float32 sum bit for bit, so m is the reference's m
// (oracle/bldp_oracle.c jl_pairwise_sum restates it).
//
// The tree is perfect down to level K = pw_level(n), the first level whose
// pieces ("blocks") hold <= 2048 elements; each block is one leaf (<= 1024)
// or two leaves split at its midpoint.  Leaves hold >= 512 elements once
// n > 1024.
//
// Paths (the window is read from HBM once on the first three):
//   nt <= 32    k_kurt_regs : a lane keeps its float4 column in registers and
//               runs the recipe in order: bit-identical to it.
//   33..512     k_kurt_mid  : a 64-channel tile in registers, lane = channel,
//               the 4 waves holding consecutive quarters of the spectra (any
//               channel alignment or step).  The Float32 sum runs down the
//               registers wave after wave; z, z2 and the Float64 sums follow
//               the recipe, the 4 partial sums are added in wave order.
//               k_kurt_mid2 (float4-column windows up to 384 spectra): the
//               same with 128 channels, two per lane, and 8 waves.
//   > 512       k_kurt_leaf : one wave per (leaf, 256 channels) streams the
//               leaf once: its sequential Float32 sum, and Float64 power sums
//               about its first spectrum, moved to the leaf's own mean.
//               k_kurt_tree / k_kurt_final_{t,w} add the leaf sums up Julia's
//               tree (-> m) and merge the central moments pairwise
//               (Chan et al. / Pebay), then move them from the exact mean to m.
//               The only difference from the recipe: z^2 and z^4 are exact
//               (Float64) instead of rounded to Float32 (relative 2^-24 per
//               term, averaging out); overflow and underflow of the Float32
//               squares are reproduced from the row's max and min.
//               k_kurt_tile: short windows of narrow products (few leaves,
//               few channels): each leaf read whole into the registers of a
//               16-wave workgroup; the recipe itself for nt <= 1024.
//   unaligned   k_kurt_leafsum + the same tree (sum only) -> m, then the
//               recipe in a second pass (k_kurt_pass, k_kurt_fold).
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include <algorithm>

#include "bldp_impl.h"

namespace bldp {

// ---- Julia's pairwise-sum tree (host and device) --------------------------
// Level of the blocks: the first level whose nodes hold <= 2048 elements.
__host__ __device__ inline int pw_level(int64_t n) {
  int K = 0;
  while (((n + ((int64_t)1 << K) - 1) >> K) > 2048) ++K;
  return K;
}
// Node j of level L of the halving of [0, n): mapreduce_impl's
// imid = ifirst + (ilast - ifirst) >> 1 gives the left half ceil(len/2).
__host__ __device__ inline void pw_node(int64_t n, int L, int64_t j, int64_t &lo, int64_t &len) {
  lo = 0;
  len = n;
  for (int l = L - 1; l >= 0; --l) {
    const int64_t left = (len + 1) >> 1;
    if ((j >> l) & 1) {
      lo += left;
      len -= left;
    } else {
      len = left;
    }
  }
}
// Leaf slot s = 2j + h of block j: a block of <= 1024 elements is one leaf
// (slot 2j + 1 is empty), a longer one splits at its midpoint.
__host__ __device__ inline void pw_leaf(int64_t n, int K, int64_t slot, int64_t &lo,
                                        int64_t &len) {
  pw_node(n, K, slot >> 1, lo, len);
  if (len > 1024) {
    const int64_t left = (len + 1) >> 1;
    if (slot & 1) {
      lo += left;
      len -= left;
    } else {
      len = left;
    }
  } else if (slot & 1) {
    lo += len;
    len = 0;
  }
}

namespace {

constexpr int kB = 256;  // 4 waves of 64
typedef float f4v __attribute__((ext_vector_type(4)));
typedef float f2v __attribute__((ext_vector_type(2)));
// streamed input: dword alignment is all gfx950's global_load_dwordx4 needs
// (plan option unaligned_vec >= 2: windows that start off a 16-byte boundary)
typedef float f4u __attribute__((ext_vector_type(4), aligned(4)));
typedef float f2u __attribute__((ext_vector_type(2), aligned(4)));
typedef double d2v __attribute__((ext_vector_type(2)));

int64_t cdivk(int64_t a, int64_t b) { return (a + b - 1) / b; }

// the window is read once: non-temporal 16-byte loads
__device__ __forceinline__ float4 ldnt(const float *p) {
  const f4u v = __builtin_nontemporal_load(reinterpret_cast<const f4u *>(p));
  return make_float4(v.x, v.y, v.z, v.w);
}

// Pairwise update of (count, mean, M2, M3, M4) with a second set
// (Chan et al.; Pebay 2008), all central moments about their own means.
__device__ __forceinline__ void moments_merge(double &na, double &ma, double &a2, double &a3,
                                              double &a4, double nb, double mb, double b2,
                                              double b3, double b4) {
  if (nb == 0.0) return;
  if (na == 0.0) {
    na = nb; ma = mb; a2 = b2; a3 = b3; a4 = b4;
    return;
  }
  const double n = na + nb, d = mb - ma, dn = d / n, dn2 = dn * dn, nab = na * nb;
  const double m4 = a4 + b4 + d * dn2 * dn * nab * (na * na - nab + nb * nb) +
                    6.0 * dn2 * (na * na * b2 + nb * nb * a2) + 4.0 * dn * (na * b3 - nb * a3);
  const double m3 = a3 + b3 + d * dn2 * nab * (na - nb) + 3.0 * dn * (na * b2 - nb * a2);
  const double m2 = a2 + b2 + d * dn * nab;
  na = n; ma += dn * nb; a2 = m2; a3 = m3; a4 = m4;
}

// StatsBase's ratio from central moments about the exact mean `ma`: move them
// to the recipe's Float32 m = S / n (z = x - m = (x - ma) + eps).  The recipe
// squares z in Float32, so cm2 (cm4) is Inf exactly when the largest z^2 (z^4)
// overflows and 0 when every one underflows; the largest |x - m| comes from
// the row's max or min.
__device__ __forceinline__ double kurt_ratio(int64_t nt, float S, double ma, double a2,
                                             double a3, double a4, float hi, float lo) {
  const float m = S / (float)nt;  // mean(v): Float32 sum / length
  const double n = (double)nt, eps = ma - (double)m, e2 = eps * eps;
  double cm2 = (a2 + n * e2) / n;
  double cm4 = (a4 + 4.0 * eps * a3 + 6.0 * e2 * a2 + n * e2 * e2) / n;
  const float zh = hi - m, zl = lo - m;
  const float h2 = zh * zh, l2 = zl * zl, h4 = h2 * h2, l4 = l2 * l2;
  if (isinf(h2) || isinf(l2))
    cm2 = INFINITY;
  else if (h2 == 0.0f && l2 == 0.0f)
    cm2 = 0.0;
  if (isinf(h4) || isinf(l4))
    cm4 = INFINITY;
  else if (h4 == 0.0f && l4 == 0.0f)
    cm4 = 0.0;
  return (cm4 / (cm2 * cm2)) - 3.0;
}

// ---------------------------------------------------------------------------
// nt <= NTMAX (<= 32): each lane keeps its float4 column of every spectrum in
// registers and runs the recipe in the recipe's own order, so the result is
// bit-identical to it.  EXACT (nt == NTMAX, e.g. the 16-spectrum 0000
// product) is straight-line code: all NTMAX loads issue back to back.
// (plan option "kurt_exact": 1 = use the exact-count instantiation).  The
// wave's 256 Float64 results go through LDS so every nt store instruction
// writes 1 KiB contiguous (+2.5% on the 0000 band against each lane's 32 B as
// two nt 16-byte stores).
template <int NTMAX, bool EXACT>
__global__ __launch_bounds__(kB) void k_kurt_regs(const KurtArgs k) {
  const int64_t ncols = k.nc / 4;
  const int64_t ctiles = (ncols + kB - 1) / kB;
  const int64_t b = blockIdx.x;
  const int64_t ib = b / ctiles, col = (b % ctiles) * kB + threadIdx.x;
  if (col >= ncols) return;
  const int bank = (int)(ib / k.ni);
  const int64_t i = ib - (int64_t)bank * k.ni;
  const float *p = k.in[bank] + k.in_off + i * k.in_ld_i + 4 * col;
  const int nt = EXACT ? NTMAX : (int)k.nt;
  const int64_t ld = k.in_ld_t;
  float4 v[NTMAX];
#pragma unroll
  for (int t = 0; t < NTMAX; ++t)
    if (EXACT || t < nt) v[t] = ldnt(p + t * ld);
  // Base.sum: sequential Float32 from the first element (nt <= 1024)
  f2v sa = {v[0].x, v[0].y}, sb = {v[0].z, v[0].w};
#pragma unroll
  for (int t = 1; t < NTMAX; ++t)
    if (EXACT || t < nt) {
      sa += f2v{v[t].x, v[t].y};
      sb += f2v{v[t].z, v[t].w};
    }
  const float m[4] = {sa.x / (float)nt, sa.y / (float)nt, sb.x / (float)nt, sb.y / (float)nt};
  double c2[4] = {0, 0, 0, 0}, c4[4] = {0, 0, 0, 0};
#pragma unroll
  for (int t = 0; t < NTMAX; ++t)
    if (EXACT || t < nt) {
      const float x[4] = {v[t].x, v[t].y, v[t].z, v[t].w};
#pragma unroll
      for (int w = 0; w < 4; ++w) {
        const float z = x[w] - m[w];  // StatsBase: z, z2 in Float32; Float64 moments
        const float z2 = z * z;
        c2[w] += (double)z2;
        c4[w] += (double)(z2 * z2);
      }
    }
  double r[4];
#pragma unroll
  for (int w = 0; w < 4; ++w) {
    const double cm2 = c2[w] / (double)nt, cm4 = c4[w] / (double)nt;
    r[w] = (cm4 / (cm2 * cm2)) - 3.0;
  }
  d2v *o = reinterpret_cast<d2v *>(k.out + ib * k.nc + 4 * col);
  if (ncols % 64 == 0 &&
      (reinterpret_cast<uintptr_t>(k.out + ib * k.nc) & 15) == 0) {
    // whole wave in range: transpose through this wave's 2 KiB of LDS so each
    // store instruction writes 1 KiB contiguous (lane L: doubles 2L, 2L+1 of
    // the wave's 256 outputs, then 128 + 2L, 129 + 2L)
    __shared__ d2v st[4][128];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    st[wave][2 * lane] = d2v{r[0], r[1]};
    st[wave][2 * lane + 1] = d2v{r[2], r[3]};
    __builtin_amdgcn_wave_barrier();
    const d2v a0 = st[wave][lane], a1 = st[wave][64 + lane];
    d2v *ow = reinterpret_cast<d2v *>(k.out + ib * k.nc + 4 * (col - lane));
    __builtin_nontemporal_store(a0, ow + lane);
    __builtin_nontemporal_store(a1, ow + 64 + lane);
  } else if ((reinterpret_cast<uintptr_t>(o) & 15) == 0) {
    __builtin_nontemporal_store(d2v{r[0], r[1]}, o);
    __builtin_nontemporal_store(d2v{r[2], r[3]}, o + 1);
  } else {
    double *od = k.out + ib * k.nc + 4 * col;
#pragma unroll
    for (int w = 0; w < 4; ++w) od[w] = r[w];
  }
}

// ---------------------------------------------------------------------------
// 32 < nt <= 4*NR (<= 512, one leaf), any window: a workgroup holds 64
// channels x nt spectra in registers, lane = channel, wave w = the spectra
// [w*nt/4, (w+1)*nt/4); a wave-instruction reads one row's 64 channels.  The
// sequential Float32 sum runs down each lane's registers wave after wave (the
// running sum handed on through LDS), every lane doing its own channel.  Then
// z, z2 and the Float64 sums run over the registers and the 4 partial sums are
// added through LDS in wave order.
template <int NR>
__global__ __launch_bounds__(kB) void k_kurt_mid(const KurtArgs k) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t ctiles = (k.nc + 63) / 64;
  const int64_t b = blockIdx.x;
  const int64_t ib = b / ctiles, c = (b % ctiles) * 64 + lane;
  const bool valid = c < k.nc;
  const int bank = (int)(ib / k.ni);
  const int64_t i = ib - (int64_t)bank * k.ni;
  const int nt = (int)k.nt;
  const int r0 = (wave * nt) >> 2, cnt = (((wave + 1) * nt) >> 2) - r0;
  const int64_t ld = k.in_ld_t;
  const float *p = k.in[bank] + k.in_off + i * k.in_ld_i + (valid ? c : 0) * k.in_cs + r0 * ld;
  float v[NR];
#pragma unroll
  for (int r = 0; r < NR; ++r)
    v[r] = (valid && r < cnt) ? __builtin_nontemporal_load(p + r * ld) : 0.0f;
  // Base.sum, sequential over the whole window (nt <= 1024 is one leaf)
  __shared__ float carry[64];
  float s = 0.0f;
#pragma unroll 1
  for (int w = 0; w < 4; ++w) {
    if (wave == w) {
      if (w > 0) s = carry[lane];
#pragma unroll
      for (int r = 0; r < NR; ++r)
        if (r < cnt) s = (w == 0 && r == 0) ? v[0] : s + v[r];  // from the first element
      carry[lane] = s;
    }
    __syncthreads();
  }
  const float m = carry[lane] / (float)nt;
  double c2 = 0.0, c4 = 0.0;
#pragma unroll
  for (int r = 0; r < NR; ++r)
    if (r < cnt) {
      const float z = v[r] - m;  // StatsBase: z, z2 in Float32; Float64 moments
      const float z2 = z * z;
      c2 += (double)z2;
      c4 += (double)(z2 * z2);
    }
  __shared__ double part[4][2][64];
  part[wave][0][lane] = c2;
  part[wave][1][lane] = c4;
  __syncthreads();
  if (wave == 0 && valid) {
    double a2 = 0.0, a4 = 0.0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      a2 += part[q][0][lane];
      a4 += part[q][1][lane];
    }
    const double cm2 = a2 / (double)nt, cm4 = a4 / (double)nt;
    k.out[ib * k.nc + c] = (cm4 / (cm2 * cm2)) - 3.0;
  }
}

// The same register tile with two adjacent channels per lane (one 8-byte load
// per lane: 512 contiguous bytes per wave-instruction instead of 256) and NW
// waves splitting the spectra (NW hand-offs of the running sums; the Float64
// sums are added in NW partials).  Float4-column windows whose waves hold <= 48
// spectra each (nt <= 384 with NW = 8, <= 115 VGPRs: 4 waves/SIMD).  A/B on
// MI355X against k_kurt_mid (profiles/r02/ab_kurt_mid2.json): the 0002 band
// (279 spectra) +4%, one 0002 bank +17%, a window 16 bytes off a 256-byte
// boundary +27%, 100 spectra +6%; at 512 spectra (3 waves/SIMD, one workgroup
// per CU) -18%, so longer windows stay on k_kurt_mid.
// Plan options: "kurt_mid_cpl" (2 = this kernel where it applies, 1 =
// k_kurt_mid only), "kurt_mid_small" (1 = windows of <= 64 spectra take 4
// waves; A/B, profiles/r03/ab_kfile_r03ad.json: 0002 band nt = 33 / 48 / 64
// 1.34 / 1.22 / 1.04x; nt >= 100 and one file no gain).  kMidNW waves per
// workgroup otherwise (4 and 16 measured and lost).
constexpr int kMidNW = 8;
template <int NR, int NW>
__global__ __launch_bounds__(64 * NW) void k_kurt_mid2(const KurtArgs k) {
  constexpr int TW = 128;  // channels per tile
  // wave and the per-wave spectrum counts are uniform over a wave: scalar
  // values make every `r < cnt` / `wave == w` test a scalar branch instead of
  // an exec-mask save/restore per spectrum
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t ctiles = (k.nc + TW - 1) / TW;
  const int64_t b = blockIdx.x;
  const int64_t ib = b / ctiles, c = (b % ctiles) * TW + 2 * lane;
  const bool valid = c < k.nc;  // (nc even: c + 1 < nc too)
  const int bank = (int)(ib / k.ni);
  const int64_t i = ib - (int64_t)bank * k.ni;
  const int nt = (int)k.nt;
  const int r0 = __builtin_amdgcn_readfirstlane((wave * nt) / NW);
  const int cnt = __builtin_amdgcn_readfirstlane((((wave + 1) * nt) / NW) - r0);
  const int64_t ld = k.in_ld_t;
  const float *p = k.in[bank] + k.in_off + i * k.in_ld_i + (valid ? c : 0) + r0 * ld;
  f2v v[NR];
#pragma unroll
  for (int r = 0; r < NR; ++r)
    v[r] = (valid && r < cnt) ? __builtin_nontemporal_load(reinterpret_cast<const f2u *>(p + r * ld))
                              : f2v{0.0f, 0.0f};
  // Base.sum, sequential over the whole window, wave after wave
  __shared__ f2v carry[64];
  f2v s = {0.0f, 0.0f};
#pragma unroll 1
  for (int w = 0; w < NW; ++w) {
    if (wave == w) {
      if (w > 0) s = carry[lane];
#pragma unroll
      for (int r = 0; r < NR; ++r)
        if (r < cnt) s = (w == 0 && r == 0) ? v[0] : s + v[r];  // from the first element
      carry[lane] = s;
    }
    __syncthreads();
  }
  const f2v sm = carry[lane];
  const f2v mv = {sm.x / (float)nt, sm.y / (float)nt};
  double a2 = 0.0, a4 = 0.0, b2 = 0.0, b4 = 0.0;
#pragma unroll
  for (int r = 0; r < NR; ++r)
    if (r < cnt) {
      // StatsBase: Float32 z, z2 (and z2*z2) for both channels at once
      // (v_pk_add_f32 / v_pk_mul_f32), Float64 moments
      const f2v z = v[r] - mv;
      const f2v q = z * z;
      const f2v q2 = q * q;
      a2 += (double)q.x;
      a4 += (double)q2.x;
      b2 += (double)q.y;
      b4 += (double)q2.y;
    }
  __shared__ double part[NW][4][64];
  part[wave][0][lane] = a2;
  part[wave][1][lane] = a4;
  part[wave][2][lane] = b2;
  part[wave][3][lane] = b4;
  __syncthreads();
  if (wave == 0 && valid) {
    double x2 = 0.0, x4 = 0.0, y2 = 0.0, y4 = 0.0;
#pragma unroll
    for (int q = 0; q < NW; ++q) {
      x2 += part[q][0][lane];
      x4 += part[q][1][lane];
      y2 += part[q][2][lane];
      y4 += part[q][3][lane];
    }
    const double n = (double)nt;
    const double k0 = ((x4 / n) / ((x2 / n) * (x2 / n))) - 3.0;
    const double k1 = ((y4 / n) / ((y2 / n) * (y2 / n))) - 3.0;
    double *o = k.out + ib * k.nc + c;
    if ((reinterpret_cast<uintptr_t>(o) & 15) == 0) {
      *reinterpret_cast<d2v *>(o) = d2v{k0, k1};
    } else {
      o[0] = k0;
      o[1] = k1;
    }
  }
}

// ---------------------------------------------------------------------------
// nt > 512: one wave per (leaf slot, 64 columns of W channels, bank x IF
// row).  Each lane streams its column down the leaf (<= 1024 spectra, B
// spectra per batch, the next batch's loads in flight while one is
// processed):
//   * the leaf's sequential Float32 sum (Base.mapreduce_impl's inner loop),
//   * max and min,
//   * Float64 power sums of d = x - c about the leaf's first spectrum c.  Any
//     |c - mean| is at most the largest deviation, which also bounds M4 from
//     below, so moving the sums to the leaf's mean loses at most ~len ulps.
// Writes the leaf's (mean, M2, M3, M4) and (sum, max, min), W contiguous
// values per lane per quantity.
//   kLeafB  spectra per batch (4: +1% on the band, +3% on one bank against 8;
//           the next batch's loads issued before this batch is processed lost
//           2%, wave caps of 2 or 3 per SIMD 1%: profiles/r02/ab_kurt_leaf_variants.json)
//   kLeafW  channels per lane (4: 16-byte loads, 1 KiB per wave-instruction;
//           2 or 1: -4 .. -5% on the band)
// Plan option "kurt_leaf_narrow": plans whose leaves would give fewer than
// this many waves per CU at kLeafW channels per lane take one channel per
// lane (4x the waves) and kLeafNB spectra per batch: short windows of narrow
// products (0001: 512 channels, nt = 513..8192 had 32-128 waves on the chip);
// 0 = never.  Each channel's arithmetic is unchanged.
constexpr int kLeafB = 4, kLeafW = 4, kLeafNB = 16;

template <int W>
__device__ __forceinline__ void ldw(const float *p, float (&x)[W]) {
  if constexpr (W == 4) {
    const f4u v = __builtin_nontemporal_load(reinterpret_cast<const f4u *>(p));
    x[0] = v.x; x[1] = v.y; x[2] = v.z; x[3] = v.w;
  } else if constexpr (W == 2) {
    const f2u v = __builtin_nontemporal_load(reinterpret_cast<const f2u *>(p));
    x[0] = v.x; x[1] = v.y;
  } else {
    x[0] = __builtin_nontemporal_load(p);
  }
}

template <int W>
struct LeafAcc {
  float s[W];  // Float32 sums
  float hi[W], lo[W];
  double c[W], a1[W], a2[W], a3[W], a4[W];
};
template <int W>
__device__ __forceinline__ void leaf_step(LeafAcc<W> &A, const float (&x)[W]) {
#pragma unroll
  for (int w = 0; w < W; ++w) {
    A.s[w] += x[w];
    A.hi[w] = fmaxf(A.hi[w], x[w]);
    A.lo[w] = fminf(A.lo[w], x[w]);
    const double d = (double)x[w] - A.c[w], d2 = d * d;
    A.a1[w] += d;
    A.a2[w] += d2;
    A.a3[w] = fma(d2, d, A.a3[w]);
    A.a4[w] = fma(d2, d2, A.a4[w]);
  }
}

template <int W, typename T>
__device__ __forceinline__ void stw(T *p, const T (&v)[W]) {
  if constexpr (W == 4 && sizeof(T) == 4) {
    *reinterpret_cast<f4v *>(p) = f4v{v[0], v[1], v[2], v[3]};
  } else if constexpr (W >= 2) {
    typedef T t2 __attribute__((ext_vector_type(2)));
#pragma unroll
    for (int w = 0; w < W; w += 2) *reinterpret_cast<t2 *>(p + w) = t2{v[w], v[w + 1]};
  } else {
    p[0] = v[0];
  }
}

// The leaf's (mean, M2, M3, M4) about its own mean, from the power sums about
// its first spectrum c, and its (sum, max, min).
template <int W>
__device__ __forceinline__ void leaf_store(const KurtArgs &k, const LeafAcc<W> &A, int64_t row,
                                           int64_t col, int64_t slot, int64_t len) {
  const int64_t n = k.nrow * k.nc, e = row * k.nc + W * col;
  const double cnt = (double)len;
  double mo[4][W];
#pragma unroll
  for (int w = 0; w < W; ++w) {
    const double dl = A.a1[w] / cnt, dl2 = dl * dl;
    mo[0][w] = A.c[w] + dl;
    mo[1][w] = A.a2[w] - A.a1[w] * dl;
    mo[2][w] = A.a3[w] - 3.0 * dl * A.a2[w] + 2.0 * cnt * dl2 * dl;
    mo[3][w] = A.a4[w] - 4.0 * dl * A.a3[w] + 6.0 * dl2 * A.a2[w] - 3.0 * cnt * dl2 * dl2;
  }
#pragma unroll
  for (int q = 0; q < 4; ++q) stw<W, double>(k.pm + (q * k.nslot + slot) * n + e, mo[q]);
  stw<W, float>(k.pf + slot * n + e, A.s);
  stw<W, float>(k.pf + (k.nslot + slot) * n + e, A.hi);
  stw<W, float>(k.pf + (2 * k.nslot + slot) * n + e, A.lo);
}

template <int W, int B>
__global__ __launch_bounds__(kB) void k_kurt_leaf(const KurtArgs k) {
  const int lane = threadIdx.x & 63;
  const int64_t u = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int64_t seg = u % k.nseg, r = u / k.nseg;
  const int64_t slot = r % k.nslot, row = r / k.nslot;
  const int64_t col = seg * 64 + lane;
  if (row >= k.nrow || col >= k.nc / W) return;
  int64_t t0, len;
  pw_leaf(k.nt, k.K, slot, t0, len);
  if (len <= 0) return;
  const int bank = (int)(row / k.ni);
  const int64_t i = row - (int64_t)bank * k.ni;
  const int64_t ld = k.in_ld_t;
  const float *p = k.in[bank] + k.in_off + i * k.in_ld_i + W * col + t0 * ld;
  LeafAcc<W> A;
  {
    float x0[W];
    ldw<W>(p, x0);
#pragma unroll
    for (int w = 0; w < W; ++w) {
      A.s[w] = A.hi[w] = A.lo[w] = x0[w];  // the sum starts from the first element
      A.c[w] = (double)x0[w];
      A.a1[w] = A.a2[w] = A.a3[w] = A.a4[w] = 0.0;
    }
  }
  p += ld;
  const int64_t rem = len - 1, nb = rem / B;
  float cur[B][W];
  if (nb > 0) {
#pragma unroll
    for (int q = 0; q < B; ++q) ldw<W>(p + q * ld, cur[q]);
  }
  for (int64_t bt = 0; bt < nb; ++bt) {
    p += B * ld;
#pragma unroll
    for (int q = 0; q < B; ++q) leaf_step<W>(A, cur[q]);
    if (bt + 1 < nb) {
#pragma unroll
      for (int q = 0; q < B; ++q) ldw<W>(p + q * ld, cur[q]);
    }
  }
  const int tail = (int)(rem - nb * B);
  if (tail > 0) {
#pragma unroll
    for (int q = 0; q < B; ++q)
      if (q < tail) ldw<W>(p + q * ld, cur[q]);
#pragma unroll
    for (int q = 0; q < B; ++q)
      if (q < tail) leaf_step<W>(A, cur[q]);
  }
  leaf_store<W>(k, A, row, col, slot, len);
}

// ---------------------------------------------------------------------------
// Leaves read whole into registers: one workgroup of kTileW waves per (64/Q
// channels, leaf, bank x IF row).  Wave w holds the spectra [w*len/kTileW,
// (w+1)*len/kTileW) of the leaf (<= 64: leaves hold <= 1024), split into Q
// consecutive pieces over Q (1 or 2) groups of 64/Q lanes (lane = piece *
// 64/Q + channel).  Every load of the leaf is in flight at once, where a streaming
// lane of k_kurt_leaf waits one memory round trip per batch: short windows of
// narrow products (0001: 512 channels, nt = 513..8192) are a few leaves deep
// and have too few lanes to hide that.  Q > 1 spreads a leaf's channels over
// Q times the workgroups (the bytes a CU can have in flight bound these
// launches).  The sequential Float32 sum runs down the registers piece after
// piece (handed on to the next lane group by a shuffle) and wave after wave
// (through LDS), as in k_kurt_mid.
//   RECIPE  (nt <= 1024, one leaf): then StatsBase's recipe over the
//           registers (Float32 m, z, z2; Float64 moments; partials added in
//           spectrum order) -> the excess kurtosis, no tree.
//   !RECIPE the leaf's partials for the tree: (sum, max, min) and (mean,
//           M2, M3, M4) about the leaf's own Float64 mean, both passes over
//           the registers.
// Plan option "kurt_leaf_tile": 1 (default) = this kernel for the plans that
// would take one channel per lane on k_kurt_leaf ("kurt_leaf_narrow") and fit
// one workgroup per CU: Q = 2 if that many fit, else Q = 1, else the streamed
// leaf (A/B, profiles/r03/ab_ktile_r03ab.json: at 2-4 workgroups per CU the
// streamed lanes win, and Q = 4 lost to Q = 2 everywhere); 2 = every leaf plan
// (Q = 2); 0 = never.
constexpr int kTileW = 16;

template <int Q, bool RECIPE>
__global__ __launch_bounds__(64 * kTileW) void k_kurt_tile(const KurtArgs k) {
  constexpr int CH = 64 / Q, NR = 1024 / kTileW / Q;  // channels, registers per lane
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int grp = lane / CH, ch = lane % CH;
  const int64_t ctiles = (k.nc + CH - 1) / CH;
  const int64_t b = blockIdx.x;
  const int64_t r = b / ctiles, c = (b % ctiles) * CH + ch;
  const int64_t slot = RECIPE ? 0 : r % k.nslot, row = RECIPE ? r : r / k.nslot;
  const bool valid = c < k.nc;
  int64_t t0 = 0, len = k.nt;
  if (!RECIPE) pw_leaf(k.nt, k.K, slot, t0, len);
  if (len <= 0) return;  // (uniform over the workgroup)
  const int bank = (int)(row / k.ni);
  const int64_t i = row - (int64_t)bank * k.ni;
  const int ln = (int)len;
  const int r0 = __builtin_amdgcn_readfirstlane((wave * ln) / kTileW);
  const int cnt = __builtin_amdgcn_readfirstlane(((wave + 1) * ln) / kTileW - r0);
  const int g0 = (grp * cnt) / Q, gn = ((grp + 1) * cnt) / Q - g0;  // this lane's piece
  const int64_t ld = k.in_ld_t;
  // lanes past the window read channel 0 of the row (results not stored)
  const float *p =
      k.in[bank] + k.in_off + i * k.in_ld_i + (valid ? c : 0) * k.in_cs + (t0 + r0 + g0) * ld;
  float v[NR];
#pragma unroll
  for (int q = 0; q < NR; ++q) v[q] = q < gn ? __builtin_nontemporal_load(p + q * ld) : 0.0f;
  // the leaf's sequential Float32 sum, from its first element
  __shared__ float carry[CH];
  float s = 0.0f;
#pragma unroll 1
  for (int w = 0; w < kTileW; ++w) {
    if (wave == w) {
      if (w > 0) s = carry[ch];
#pragma unroll
      for (int g = 0; g < Q; ++g) {
        if (grp == g) {
#pragma unroll
          for (int q = 0; q < NR; ++q)
            if (q < gn) s = (w == 0 && g == 0 && q == 0) ? v[0] : s + v[q];
        }
        if (g + 1 < Q) s = __shfl_up(s, CH, 64);  // group g's sums to group g + 1
      }
      if (grp == Q - 1) carry[ch] = s;
    }
    __syncthreads();
  }
  const float S = carry[ch];
  if constexpr (RECIPE) {
    const float m = S / (float)ln;  // mean(v): Float32 sum / length
    double c2 = 0.0, c4 = 0.0;
#pragma unroll
    for (int q = 0; q < NR; ++q)
      if (q < gn) {
        const float z = v[q] - m;  // StatsBase: z, z2 in Float32; Float64 moments
        const float z2 = z * z;
        c2 += (double)z2;
        c4 += (double)(z2 * z2);
      }
    __shared__ double part[kTileW][2][64];
    part[wave][0][lane] = c2;
    part[wave][1][lane] = c4;
    __syncthreads();
    if (wave == 0 && grp == 0 && valid) {
      double a2 = 0.0, a4 = 0.0;
#pragma unroll
      for (int w = 0; w < kTileW; ++w)
#pragma unroll
        for (int g = 0; g < Q; ++g) {
          a2 += part[w][0][g * CH + ch];
          a4 += part[w][1][g * CH + ch];
        }
      const double cm2 = a2 / (double)ln, cm4 = a4 / (double)ln;
      k.out[row * k.nc + c] = (cm4 / (cm2 * cm2)) - 3.0;
    }
  } else {
    // pass 1: max, min and the Float64 sum -> the leaf's mean (gn >= 8: leaves
    // of a tree hold >= 512 spectra)
    float hi = v[0], lo = v[0];
    double d1 = 0.0;
#pragma unroll
    for (int q = 0; q < NR; ++q)
      if (q < gn) {
        hi = fmaxf(hi, v[q]);
        lo = fminf(lo, v[q]);
        d1 += (double)v[q];
      }
    __shared__ double p1[kTileW][64];
    __shared__ float ph[kTileW][64], pl[kTileW][64];
    p1[wave][lane] = d1;
    ph[wave][lane] = hi;
    pl[wave][lane] = lo;
    __syncthreads();
    double tot = 0.0;  // in spectrum order: every lane of a channel agrees
#pragma unroll
    for (int w = 0; w < kTileW; ++w)
#pragma unroll
      for (int g = 0; g < Q; ++g) tot += p1[w][g * CH + ch];
    const double md = tot / (double)ln;
    // pass 2: central moments about it
    double a2 = 0.0, a3 = 0.0, a4 = 0.0;
#pragma unroll
    for (int q = 0; q < NR; ++q)
      if (q < gn) {
        const double d = (double)v[q] - md, d2 = d * d;
        a2 += d2;
        a3 = fma(d2, d, a3);
        a4 = fma(d2, d2, a4);
      }
    __shared__ double p2[kTileW][3][64];
    p2[wave][0][lane] = a2;
    p2[wave][1][lane] = a3;
    p2[wave][2][lane] = a4;
    __syncthreads();
    if (wave == 0 && grp == 0 && valid) {
      double m2 = 0.0, m3 = 0.0, m4 = 0.0;
#pragma unroll
      for (int w = 0; w < kTileW; ++w)
#pragma unroll
        for (int g = 0; g < Q; ++g) {
          m2 += p2[w][0][g * CH + ch];
          m3 += p2[w][1][g * CH + ch];
          m4 += p2[w][2][g * CH + ch];
          hi = fmaxf(hi, ph[w][g * CH + ch]);
          lo = fminf(lo, pl[w][g * CH + ch]);
        }
      const int64_t n = k.nrow * k.nc, e = row * k.nc + c;
      k.pm[slot * n + e] = md;
      k.pm[(k.nslot + slot) * n + e] = m2;
      k.pm[(2 * k.nslot + slot) * n + e] = m3;
      k.pm[(3 * k.nslot + slot) * n + e] = m4;
      k.pf[slot * n + e] = S;
      k.pf[(k.nslot + slot) * n + e] = hi;
      k.pf[(2 * k.nslot + slot) * n + e] = lo;
    }
  }
}

// Unaligned windows: one lane per (column, leaf) runs the sequential Float32
// sum of the leaf (any channel step); sums only.
__global__ __launch_bounds__(kB) void k_kurt_leafsum(const KurtArgs k) {
  const int64_t ctiles = (k.nc + kB - 1) / kB;
  int64_t b = blockIdx.x;
  const int64_t ct = b % ctiles;
  b /= ctiles;
  const int64_t slot = b % k.nslot, row = b / k.nslot;
  const int64_t c = ct * kB + threadIdx.x;
  if (row >= k.nrow || c >= k.nc) return;
  int64_t t0, len;
  pw_leaf(k.nt, k.K, slot, t0, len);
  if (len <= 0) return;
  const int bank = (int)(row / k.ni);
  const int64_t i = row - (int64_t)bank * k.ni;
  const int64_t ld = k.in_ld_t;
  const float *p = k.in[bank] + k.in_off + i * k.in_ld_i + c * k.in_cs + t0 * ld;
  float s = p[0];
  int64_t t = 1;
  for (; t + 8 <= len; t += 8) {
    float v[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) v[q] = p[(t + q) * ld];
#pragma unroll
    for (int q = 0; q < 8; ++q) s += v[q];
  }
  for (; t < len; ++t) s += p[t * ld];
  k.pf[slot * (k.nrow * k.nc) + row * k.nc + c] = s;
}

// ---- the tree: leaf sums -> m, leaf moments -> row moments ----------------
// Partials of the nodes of one level: component q of node j of output e at
// [(q * nodes + j) * n + e] (pm: mean, M2, M3, M4; pf: sum, max, min).
struct TreeIO {
  const double *pm;
  const float *pf;
  int64_t nin;   // input nodes (FIRST: leaf slots)
  double *pmo;
  float *pfo;
  int64_t nout;  // output nodes
  int L;         // level of the input nodes (FIRST: K, blocks built from leaves)
};
struct Node {
  float S, hi, lo;
  double n, m, a2, a3, a4;
};
// Input node j of output e.  FIRST: block j of leaves 2j and 2j+1
// (mapreduce_impl's op(v1, v2) = v1 + v2 for a split block).
template <bool FIRST, bool MOM>
__device__ __forceinline__ Node load_node(const KurtArgs &k, const TreeIO &io, int64_t n,
                                          int64_t e, int64_t j) {
  Node x;
  x.hi = -INFINITY;
  x.lo = INFINITY;
  x.n = x.m = x.a2 = x.a3 = x.a4 = 0.0;
  const int64_t ns = io.nin * n;  // stride between components
  if (FIRST) {
    int64_t lo0, len0, lo1, len1;
    pw_leaf(k.nt, k.K, 2 * j, lo0, len0);
    pw_leaf(k.nt, k.K, 2 * j + 1, lo1, len1);
    const int64_t s0 = 2 * j * n + e, s1 = s0 + n;
    x.S = io.pf[s0];
    if (MOM) {
      x.hi = io.pf[ns + s0];
      x.lo = io.pf[2 * ns + s0];
      x.n = (double)len0;
      x.m = io.pm[s0];
      x.a2 = io.pm[ns + s0];
      x.a3 = io.pm[2 * ns + s0];
      x.a4 = io.pm[3 * ns + s0];
    }
    if (len1 > 0) {
      x.S = x.S + io.pf[s1];
      if (MOM) {
        x.hi = fmaxf(x.hi, io.pf[ns + s1]);
        x.lo = fminf(x.lo, io.pf[2 * ns + s1]);
        moments_merge(x.n, x.m, x.a2, x.a3, x.a4, (double)len1, io.pm[s1], io.pm[ns + s1],
                      io.pm[2 * ns + s1], io.pm[3 * ns + s1]);
      }
    }
  } else {
    const int64_t s0 = j * n + e;
    x.S = io.pf[s0];
    if (MOM) {
      int64_t lo, len;
      pw_node(k.nt, io.L, j, lo, len);
      x.hi = io.pf[ns + s0];
      x.lo = io.pf[2 * ns + s0];
      x.n = (double)len;
      x.m = io.pm[s0];
      x.a2 = io.pm[ns + s0];
      x.a3 = io.pm[2 * ns + s0];
      x.a4 = io.pm[3 * ns + s0];
    }
  }
  return x;
}

// Q consecutive input nodes of one output into one node (a perfect subtree):
// the sums pairwise in tree order, the moments merged in node order.
template <int Q, bool FIRST, bool MOM>
__device__ __forceinline__ Node fold_nodes(const KurtArgs &k, const TreeIO &io, int64_t n,
                                           int64_t e, int64_t g) {
  float s[Q];
  Node acc;
  acc.hi = -INFINITY;
  acc.lo = INFINITY;
  acc.n = acc.m = acc.a2 = acc.a3 = acc.a4 = 0.0;
#pragma unroll
  for (int q = 0; q < Q; ++q) {
    const Node x = load_node<FIRST, MOM>(k, io, n, e, g * Q + q);
    s[q] = x.S;
    if (MOM) {
      acc.hi = fmaxf(acc.hi, x.hi);
      acc.lo = fminf(acc.lo, x.lo);
      moments_merge(acc.n, acc.m, acc.a2, acc.a3, acc.a4, x.n, x.m, x.a2, x.a3, x.a4);
    }
  }
#pragma unroll
  for (int w = 1; w < Q; w *= 2)
#pragma unroll
    for (int q = 0; q < Q; q += 2 * w) s[q] = s[q] + s[q + w];
  acc.S = s[0];
  return acc;
}

template <int Q, bool FIRST, bool MOM>
__global__ __launch_bounds__(kB) void k_kurt_tree(const KurtArgs k, const TreeIO io) {
  const int64_t n = k.nrow * k.nc, total = io.nout * n;
  for (int64_t x = (int64_t)blockIdx.x * kB + threadIdx.x; x < total;
       x += (int64_t)gridDim.x * kB) {
    const int64_t g = x / n, e = x - g * n;
    const Node a = fold_nodes<Q, FIRST, MOM>(k, io, n, e, g);
    const int64_t ns = io.nout * n, s0 = g * n + e;
    io.pfo[s0] = a.S;
    if (MOM) {
      io.pfo[ns + s0] = a.hi;
      io.pfo[2 * ns + s0] = a.lo;
      io.pmo[s0] = a.m;
      io.pmo[ns + s0] = a.a2;
      io.pmo[2 * ns + s0] = a.a3;
      io.pmo[3 * ns + s0] = a.a4;
    }
  }
}

// Last level, one thread per output (Q = all remaining nodes): MOM -> the
// excess kurtosis, else the Float32 mean for the two-pass path.
template <int Q, bool FIRST, bool MOM>
__global__ __launch_bounds__(kB) void k_kurt_final_t(const KurtArgs k, const TreeIO io) {
  const int64_t n = k.nrow * k.nc;
  for (int64_t e = (int64_t)blockIdx.x * kB + threadIdx.x; e < n;
       e += (int64_t)gridDim.x * kB) {
    const Node a = fold_nodes<Q, FIRST, MOM>(k, io, n, e, 0);
    if (MOM)
      k.out[e] = kurt_ratio(k.nt, a.S, a.m, a.a2, a.a3, a.a4, a.hi, a.lo);
    else
      k.mean[e] = a.S / (float)k.nt;
  }
}

// Last level, one wave per output, lane j holding node j (<= 64 nodes): an xor
// butterfly over consecutive lanes is exactly the perfect tree of the sums
// (Float32 addition commutes); the moments merge the lower lane's first, so
// both lanes of a pair agree.
template <bool FIRST, bool MOM>
__global__ __launch_bounds__(kB) void k_kurt_final_w(const KurtArgs k, const TreeIO io) {
  const int lane = threadIdx.x & 63;
  const int64_t n = k.nrow * k.nc;
  const int nn = 1 << io.L;
  for (int64_t e = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); e < n;
       e += (int64_t)gridDim.x * 4) {
    Node a;
    a.S = 0.0f;
    a.hi = -INFINITY;
    a.lo = INFINITY;
    a.n = a.m = a.a2 = a.a3 = a.a4 = 0.0;
    if (lane < nn) a = load_node<FIRST, MOM>(k, io, n, e, lane);
    for (int off = 1; off < nn; off <<= 1) {
      a.S = a.S + __shfl_xor(a.S, off, 64);
      if (MOM) {
        a.hi = fmaxf(a.hi, __shfl_xor(a.hi, off, 64));
        a.lo = fminf(a.lo, __shfl_xor(a.lo, off, 64));
        const double nb = __shfl_xor(a.n, off, 64), mb = __shfl_xor(a.m, off, 64);
        const double b2 = __shfl_xor(a.a2, off, 64), b3 = __shfl_xor(a.a3, off, 64);
        const double b4 = __shfl_xor(a.a4, off, 64);
        if (lane & off) {  // the partner is the lower lane: it goes first
          double xn = nb, xm = mb, x2 = b2, x3 = b3, x4 = b4;
          moments_merge(xn, xm, x2, x3, x4, a.n, a.m, a.a2, a.a3, a.a4);
          a.n = xn; a.m = xm; a.a2 = x2; a.a3 = x3; a.a4 = x4;
        } else {
          moments_merge(a.n, a.m, a.a2, a.a3, a.a4, nb, mb, b2, b3, b4);
        }
      }
    }
    if (lane == 0) {
      if (MOM)
        k.out[e] = kurt_ratio(k.nt, a.S, a.m, a.a2, a.a3, a.a4, a.hi, a.lo);
      else
        k.mean[e] = a.S / (float)k.nt;
    }
  }
}

// ---------------------------------------------------------------------------
// Two-pass recipe for unaligned windows, given the Float32 mean: one lane per
// column, `ts` waves of a workgroup splitting the spectra of a tile (4/ts
// tiles per workgroup), 8 loads in flight, Float64 partials combined through
// LDS in wave order.  With one time chunk the ratio is written here;
// otherwise chunks are folded in a fixed order by k_kurt_fold.
// At most 4 resident waves per SIMD.
__global__ __launch_bounds__(kB) __attribute__((amdgpu_waves_per_eu(1, 4)))
void k_kurt_pass(const KurtArgs k) {
  constexpr int B = 8;  // spectra in flight per lane
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int ts = k.ts, wt = wave / ts, tsi = wave - wt * ts;
  const int64_t ctiles = (k.nc + 63) / 64, tpb = 4 / ts;
  const int64_t cblocks = (ctiles + tpb - 1) / tpb;
  int64_t b = blockIdx.x;
  const int64_t cb = b % cblocks;
  b /= cblocks;
  const int64_t ib = b % k.nrow, chunk = b / k.nrow;  // (bank, IF) row, time chunk
  const int bank = (int)(ib / k.ni);
  const int64_t i = ib - (int64_t)bank * k.ni;
  const int64_t col = (cb * tpb + wt) * 64 + lane;
  const bool valid = col < k.nc;
  const int64_t r0 = chunk * k.rows_per_chunk, r1 = min(k.nt, r0 + k.rows_per_chunk);
  const int64_t e = ib * k.nc + col;
  double a2 = 0.0, a4 = 0.0;
  if (valid) {
    const float *p = k.in[bank] + k.in_off + i * k.in_ld_i + (r0 + tsi) * k.in_ld_t + col * k.in_cs;
    const float m = k.mean[e];
    int64_t n = r1 - r0 - tsi;
    n = n > 0 ? (n + ts - 1) / ts : 0;
    const int64_t st = (int64_t)ts * k.in_ld_t;
    for (; n > 0; n -= B, p += B * st) {
      float v[B];  // predicated batch: spectra past the end read as the mean (z = 0)
#pragma unroll
      for (int u = 0; u < B; ++u) v[u] = u < n ? p[u * st] : m;
#pragma unroll
      for (int u = 0; u < B; ++u) {
        // StatsBase: z = v[i] - m; z2 = z*z (Float32); cm2 += z2; cm4 += z2*z2
        const float z = v[u] - m;
        const float z2 = z * z;
        a2 += (double)z2;
        a4 += (double)(z2 * z2);
      }
    }
  }
  if (ts > 1) {
    __shared__ double red[4][2][64];
    red[wave][0][lane] = a2;
    red[wave][1][lane] = a4;
    __syncthreads();
    if (tsi == 0)
      for (int q = 1; q < ts; ++q) {
        a2 += red[wave + q][0][lane];
        a4 += red[wave + q][1][lane];
      }
  }
  if (tsi == 0 && valid) {
    const int64_t n = k.nrow * k.nc;
    if (k.nchunk == 1) {
      const double cm2 = a2 / (double)k.nt, cm4 = a4 / (double)k.nt;
      k.out[e] = (cm4 / (cm2 * cm2)) - 3.0;
    } else {
      k.ws_mom[(chunk * 2) * n + e] = a2;
      k.ws_mom[(chunk * 2 + 1) * n + e] = a4;
    }
  }
}

// Fold the time-chunk partials of every output, chunks in order.
__global__ __launch_bounds__(kB) void k_kurt_fold(const KurtArgs k) {
  const int64_t n = k.nrow * k.nc;
  for (int64_t e = (int64_t)blockIdx.x * kB + threadIdx.x; e < n;
       e += (int64_t)gridDim.x * kB) {
    double a = 0.0, c = 0.0;
    for (int ch = 0; ch < k.nchunk; ++ch) {
      a += k.ws_mom[(ch * 2) * n + e];
      c += k.ws_mom[(ch * 2 + 1) * n + e];
    }
    const double cm2 = a / (double)k.nt, cm4 = c / (double)k.nt;
    k.out[e] = (cm4 / (cm2 * cm2)) - 3.0;
  }
}

__global__ __launch_bounds__(kB) void k_fill_nan(double *out, int64_t n) {
  for (int64_t e = (int64_t)blockIdx.x * kB + threadIdx.x; e < n; e += (int64_t)gridDim.x * kB)
    out[e] = NAN;
}

// ---- host side -------------------------------------------------------------
// spectra per wave of the largest k_kurt_mid instantiation (windows up to 4 x
// this many spectra use it)
constexpr int kMidNR = 128;

enum KPath { KP_REGS = 0, KP_MID = 1, KP_LEAF = 2, KP_TWOPASS = 3 };

int path_of(const KurtArgs &k) {
  if (k.vec && k.nt <= 32) return KP_REGS;
  if (k.nt <= 4 * kMidNR) return KP_MID;  // any channel alignment and step
  if (k.vec) return KP_LEAF;
  return KP_TWOPASS;
}

// Workspace regions: A holds the leaf partials, B the first tree level's;
// later tree levels alternate between them (each is smaller than A).
struct KLayout {
  size_t a_pm, a_pf, b_pm, b_pf, mean, mom, total;
};
size_t up256(size_t b) { return (b + 255) & ~(size_t)255; }
KLayout layout(const KurtArgs &k) {
  KLayout L{};
  const size_t n = (size_t)k.nrow * k.nc, ns = (size_t)k.nslot, nb = ns / 2;
  const int p = path_of(k);
  size_t off = 0;
  auto take = [&](size_t bytes) {
    const size_t o = off;
    off += up256(bytes);
    return o;
  };
  if (p == KP_LEAF) {
    L.a_pm = take(4 * ns * n * sizeof(double));
    L.a_pf = take(3 * ns * n * sizeof(float));
    L.b_pm = take(4 * nb * n * sizeof(double));
    L.b_pf = take(3 * nb * n * sizeof(float));
  } else if (p == KP_TWOPASS) {
    L.a_pf = take(ns * n * sizeof(float));
    L.b_pf = take(nb * n * sizeof(float));
    L.mean = take(n * sizeof(float));
    L.mom = k.nchunk > 1 ? take(2 * (size_t)k.nchunk * n * sizeof(double)) : off;
  }
  L.total = off;
  return L;
}

template <bool MOM>
hipError_t launch_tree_pass(const KurtArgs &k, const TreeIO &io, int q, bool first, hipStream_t s) {
  const int64_t total = io.nout * k.nrow * k.nc;
  const dim3 g((unsigned)std::min<int64_t>(cdivk(total, kB), 1 << 20)), b(kB);
#define BLDP_TREE(Q)                                                          \
  if (first)                                                                  \
    hipLaunchKernelGGL((k_kurt_tree<Q, true, MOM>), g, b, 0, s, k, io);       \
  else                                                                        \
    hipLaunchKernelGGL((k_kurt_tree<Q, false, MOM>), g, b, 0, s, k, io);
  switch (q) {
    case 1: BLDP_TREE(2) break;
    case 2: BLDP_TREE(4) break;
    case 3: BLDP_TREE(8) break;
    case 4: BLDP_TREE(16) break;
    default: return hipErrorInvalidValue;
  }
#undef BLDP_TREE
  return hipGetLastError();
}

template <bool MOM>
hipError_t launch_final(const KurtArgs &k, const TreeIO &io, bool first, hipStream_t s) {
  const int64_t n = k.nrow * k.nc;
  const dim3 b(kB);
  if (io.L >= 3) {
    const dim3 g((unsigned)std::min<int64_t>(cdivk(n, 4), 1 << 20));
    if (first)
      hipLaunchKernelGGL((k_kurt_final_w<true, MOM>), g, b, 0, s, k, io);
    else
      hipLaunchKernelGGL((k_kurt_final_w<false, MOM>), g, b, 0, s, k, io);
    return hipGetLastError();
  }
  const dim3 g((unsigned)std::min<int64_t>(cdivk(n, kB), 1 << 20));
#define BLDP_FINAL(Q)                                                         \
  if (first)                                                                  \
    hipLaunchKernelGGL((k_kurt_final_t<Q, true, MOM>), g, b, 0, s, k, io);    \
  else                                                                        \
    hipLaunchKernelGGL((k_kurt_final_t<Q, false, MOM>), g, b, 0, s, k, io);
  switch (io.L) {
    case 0: BLDP_FINAL(1) break;
    case 1: BLDP_FINAL(2) break;
    case 2: BLDP_FINAL(4) break;
    default: return hipErrorInvalidValue;
  }
#undef BLDP_FINAL
  return hipGetLastError();
}

// Leaf partials in region A -> the row results.  Passes of up to 4 levels
// (16 nodes per thread) run while more than 64 nodes remain; the last <= 64
// nodes go to one wave per output (or one thread when <= 4 remain).
template <bool MOM>
hipError_t launch_tree(const KurtArgs &k, char *ws, const KLayout &L, hipStream_t s) {
  double *pm[2] = {reinterpret_cast<double *>(ws + L.a_pm), reinterpret_cast<double *>(ws + L.b_pm)};
  float *pf[2] = {reinterpret_cast<float *>(ws + L.a_pf), reinterpret_cast<float *>(ws + L.b_pf)};
  TreeIO io{};
  int cur = 0;
  io.pm = pm[0];
  io.pf = pf[0];
  io.nin = k.nslot;
  io.L = k.K;
  bool first = true;
  while (io.L > 6) {
    const int q = std::min(4, io.L - 6);
    io.nout = (int64_t)1 << (io.L - q);
    io.pmo = pm[1 - cur];
    io.pfo = pf[1 - cur];
    hipError_t e = launch_tree_pass<MOM>(k, io, q, first, s);
    if (e != hipSuccess) return e;
    cur = 1 - cur;
    io.pm = pm[cur];
    io.pf = pf[cur];
    io.nin = io.nout;
    io.L -= q;
    first = false;
  }
  return launch_final<MOM>(k, io, first, s);
}

}  // namespace

// Dynamic LDS per workgroup of k_kurt_leaf / k_kurt_mid2 as a cap on the
// workgroups resident per CU (as kIlShm in kernels.hip); 0 = no cap: the leaf
// at 2 / 4 per CU within +-1% on every kurtosis shape but one, k_kurt_mid2 at
// 2 per CU 62% slower on cfg2 (round 5, profiles/r05/ab_kurt_r05g2.json).
constexpr unsigned kKurtLeafShm = 0, kKurtMidShm = 0;
// k_kurt_regs (<= 32 spectra: a lane's whole float4 column in flight at once,
// 16-32 x 16 B per lane): 2 workgroups per CU for windows of 12-16 spectra
// (48-64 KiB of loads a workgroup), uncapped otherwise.  Round 5 A/B
// (profiles/r05/ab_kregs_r05h.json, one process, one box), time relative to
// uncapped: the 0000 band nt = 12 / 16 0.946 / 0.969, one 0000 bank nt = 16
// 0.920, c0 = 1 0.974, the 0002 band nt = 16 0.965; but nt = 4 / 8 1.21 /
// 1.09 (there the Float64 outputs are 1/2 - 1/4 of the traffic) and nt = 32
// 1.02 (3 / 4 per CU: within +-3% either way).  Re-run on another box
// (ab_kregs_r05s.json, against this cap): uncapped 1.004 on the band, 1.038 on
// one bank; 1 per CU 1.15-1.53; 3 per CU within +-1%.
constexpr unsigned kKurtRegsShm = 65536;
constexpr int64_t kKurtRegsCapLo = 12, kKurtRegsCapHi = 16;

void plan_kurtosis(KurtArgs &k, int num_cus) {
  k.K = pw_level(std::max<int64_t>(k.nt, 1));
  k.nslot = (int64_t)2 << k.K;
  k.leafw = kLeafW;
  const int64_t narrow = opt(OPT_KURT_LEAF_NARROW);
  if (narrow > 0 && kLeafW > 1 && k.nrow * k.nslot * cdivk(k.nc / kLeafW, 64) < num_cus * narrow)
    k.leafw = 1;
  k.leaftile = 0;  // lane groups per channel of k_kurt_tile; 0 = streamed leaves
  if (opt(OPT_KURT_LEAF_TILE) == 1 && k.leafw == 1) {
    const int64_t units = k.nrow * (k.nt <= 1024 ? 1 : k.nslot);  // leaves x rows
    if (units * cdivk(k.nc, 32) <= num_cus)
      k.leaftile = 2;
    else if (units * cdivk(k.nc, 64) <= num_cus)
      k.leaftile = 1;
  }
  k.nseg = cdivk(k.nc / k.leafw, 64);
  // two-pass z pass: waves splitting the spectra of a tile, >= 16 spectra per wave
  k.ts = 1;
  while (k.ts < 4 && k.nt >= (int64_t)32 * k.ts) k.ts *= 2;
  const int64_t tiles = cdivk(cdivk(k.nc, 64), 4 / k.ts) * k.nrow;  // workgroups
  const int64_t target = (int64_t)num_cus * 8;
  int64_t nchunk = 1;
  if (tiles > 0 && tiles < target)  // (empty windows: no split)
    nchunk = std::min<int64_t>(cdivk(target, tiles), k.nt / (16 * k.ts));
  nchunk = std::max<int64_t>(nchunk, 1);
  k.rows_per_chunk = std::max<int64_t>(1, cdivk(k.nt, nchunk));
  k.nchunk = (int32_t)std::max<int64_t>(1, cdivk(k.nt, k.rows_per_chunk));
}

int kurtosis_path(const KurtArgs &k) { return path_of(k); }

size_t kurtosis_ws_bytes(const KurtArgs &k) { return layout(k).total; }

hipError_t launch_kurtosis(KurtArgs &k, char *ws, hipStream_t s) {
  const int64_t n = k.nrow * k.nc;
  if (n == 0) return hipSuccess;
  const dim3 block(kB);
  const int p = path_of(k);
  if (k.nt == 0) {  // mean of nothing: StatsBase gives 0/0 - 3 = NaN
    const unsigned g = (unsigned)std::min<int64_t>(cdivk(n, kB), 16384);
    hipLaunchKernelGGL(k_fill_nan, dim3(g), block, 0, s, k.out, n);
    return hipGetLastError();
  }
  const int64_t ncols = k.nc / 4;
  if (p == KP_REGS) {
    const dim3 g1((unsigned)(cdivk(ncols, kB) * k.nrow));
    const bool exact = opt(OPT_KURT_EXACT) != 0;
    const unsigned shm = k.nt >= kKurtRegsCapLo && k.nt <= kKurtRegsCapHi ? kKurtRegsShm : 0;
    if (exact && k.nt == 16)
      hipLaunchKernelGGL((k_kurt_regs<16, true>), g1, block, shm, s, k);
    else if (exact && k.nt == 32)
      hipLaunchKernelGGL((k_kurt_regs<32, true>), g1, block, shm, s, k);
    else if (k.nt <= 16)
      hipLaunchKernelGGL((k_kurt_regs<16, false>), g1, block, shm, s, k);
    else
      hipLaunchKernelGGL((k_kurt_regs<32, false>), g1, block, shm, s, k);
    return hipGetLastError();
  }
  if (p == KP_MID && opt(OPT_KURT_MID_CPL) == 2 && k.vec && cdivk(k.nt, 8) <= 48) {
    constexpr int NW = kMidNW;
    const dim3 g1((unsigned)(cdivk(k.nc, 128) * k.nrow)), b2(64 * NW);
    if (opt(OPT_KURT_MID_SMALL) && k.nt <= 64) {  // (33..64 here) 4 waves of <= 16 spectra
      hipLaunchKernelGGL((k_kurt_mid2<16, 4>), g1, dim3(256), 0, s, k);
      return hipGetLastError();
    }
    // registers sized to a wave's spectra, 8 at a time (occupancy: 113 VGPRs
    // at 48 spectra = 4 waves/SIMD, 80 at 32 = 6, 48 at 16 = 8)
    switch (cdivk(cdivk(k.nt, NW), 8)) {
#define BLDP_MID2(NR) hipLaunchKernelGGL((k_kurt_mid2<NR, NW>), g1, b2, kKurtMidShm, s, k); break;
      case 1: BLDP_MID2(8)
      case 2: BLDP_MID2(16)
      case 3: BLDP_MID2(24)
      case 4: BLDP_MID2(32)
      case 5: BLDP_MID2(40)
      case 6: BLDP_MID2(48)
#undef BLDP_MID2
      default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
  }
  if (p == KP_MID) {  // registers sized to the quarter window, 16 spectra at a time
    const dim3 g1((unsigned)(cdivk(k.nc, 64) * k.nrow));
    switch (cdivk(cdivk(k.nt, 4), 16)) {
      case 1: hipLaunchKernelGGL(k_kurt_mid<16>, g1, block, 0, s, k); break;
      case 2: hipLaunchKernelGGL(k_kurt_mid<32>, g1, block, 0, s, k); break;
      case 3: hipLaunchKernelGGL(k_kurt_mid<48>, g1, block, 0, s, k); break;
      case 4: hipLaunchKernelGGL(k_kurt_mid<64>, g1, block, 0, s, k); break;
      case 5: hipLaunchKernelGGL(k_kurt_mid<80>, g1, block, 0, s, k); break;
      case 6: hipLaunchKernelGGL(k_kurt_mid<96>, g1, block, 0, s, k); break;
      case 7: hipLaunchKernelGGL(k_kurt_mid<112>, g1, block, 0, s, k); break;
      default: hipLaunchKernelGGL(k_kurt_mid<128>, g1, block, 0, s, k); break;
    }
    return hipGetLastError();
  }
  const KLayout L = layout(k);
  if (p == KP_LEAF) {
    k.pm = reinterpret_cast<double *>(ws + L.a_pm);
    k.pf = reinterpret_cast<float *>(ws + L.a_pf);
    if (k.leaftile) {
      const bool recipe = k.nt <= 1024;  // one leaf: the recipe itself, no tree
      const int Q = k.leaftile;
      const dim3 gt((unsigned)(cdivk(k.nc, 64 / Q) * k.nrow * (recipe ? 1 : k.nslot))), bt(64 * kTileW);
      if (recipe) {
        if (Q == 2)
          hipLaunchKernelGGL((k_kurt_tile<2, true>), gt, bt, 0, s, k);
        else
          hipLaunchKernelGGL((k_kurt_tile<1, true>), gt, bt, 0, s, k);
        return hipGetLastError();
      }
      if (Q == 2)
        hipLaunchKernelGGL((k_kurt_tile<2, false>), gt, bt, 0, s, k);
      else
        hipLaunchKernelGGL((k_kurt_tile<1, false>), gt, bt, 0, s, k);
      hipError_t e = hipGetLastError();
      if (e != hipSuccess) return e;
      return launch_tree<true>(k, ws, L, s);
    }
    const dim3 g1((unsigned)cdivk(k.nrow * k.nslot * k.nseg, 4));
    if (k.leafw == 1)
      hipLaunchKernelGGL((k_kurt_leaf<1, kLeafNB>), g1, block, kKurtLeafShm, s, k);
    else
      hipLaunchKernelGGL((k_kurt_leaf<kLeafW, kLeafB>), g1, block, kKurtLeafShm, s, k);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    return launch_tree<true>(k, ws, L, s);
  }
  // unaligned: Float32 mean through the tree, then the z pass
  k.pf = reinterpret_cast<float *>(ws + L.a_pf);
  k.mean = reinterpret_cast<float *>(ws + L.mean);
  k.ws_mom = reinterpret_cast<double *>(ws + L.mom);
  {
    const dim3 g0((unsigned)(cdivk(k.nc, kB) * k.nrow * k.nslot));
    hipLaunchKernelGGL(k_kurt_leafsum, g0, block, 0, s, k);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    e = launch_tree<false>(k, ws, L, s);
    if (e != hipSuccess) return e;
  }
  const dim3 grid((unsigned)(cdivk(cdivk(k.nc, 64), 4 / k.ts) * k.nrow * k.nchunk));
  hipLaunchKernelGGL(k_kurt_pass, grid, block, 0, s, k);
  if (k.nchunk > 1) {
    const unsigned fg = (unsigned)std::min<int64_t>(cdivk(n, kB), 16384);
    hipLaunchKernelGGL(k_kurt_fold, dim3(fg), block, 0, s, k);
  }
  return hipGetLastError();
}

// The largest grid of the plan, for the ABI's one-launch check.
int64_t kurtosis_max_grid(const KurtArgs &k) {
  const int p = path_of(k);
  const int64_t ncols = k.nc / 4;
  switch (p) {
    case KP_REGS: return cdivk(ncols, kB) * k.nrow;
    case KP_MID: return cdivk(k.nc, 64) * k.nrow;  // (k_kurt_mid2: half of it)
    case KP_LEAF:
      if (k.leaftile) return cdivk(k.nc, 64 / k.leaftile) * k.nrow * (k.nt <= 1024 ? 1 : k.nslot);
      return cdivk(k.nrow * k.nslot * k.nseg, 4);
    default:
      return std::max(cdivk(k.nc, kB) * k.nrow * k.nslot,
                      cdivk(cdivk(k.nc, 64), 4 / k.ts) * k.nrow * k.nchunk);
  }
}

}  // namespace bldp
