// typed.hip — fqav and getkurtosis for element types other than Float32, with
// the reference's result types.
//
// The BL products are Float32, but the reference's worker functions accept
// whatever the reader returns: Blio maps SIGPROC nbits 8 / 16 to UInt8 /
// UInt16 (src/gbtworkerfunctions.jl:173), HDF5.jl returns an integer or
// Float64 dataset as such (:181-186), and fqav / getkurtosis then run Julia's
// own arithmetic on it (:16-20, :197-202):
//   * sum(reshape(A, (n, :, ...)); dims = 1) widens small integers
//     (Base.add_sum: UInt8/16/32 -> UInt64, Int8/16/32 -> Int64; 64-bit and
//     Float64 stay as they are), so every integer sum here is exact (wrapping
//     like Julia's Int64 / UInt64 on overflow) and a Float64 sum is taken in
//     the reference's order: Base's reducedim seeds zero(T) and adds
//     mapreduce_impl of the group, i.e. up to 1024 channels in sequence and
//     pairwise halves above that (jl_dimsum_f64); the time integration is fqav
//     on axis 3, so a time block's spectral sums are combined the same way;
//   * mean(...; dims = 1) is Float64 for integer and Float64 input: the
//     values converted to Float64 (Statistics' _mean_promote) summed in that
//     same order, divided by n;
//   * maximum / minimum keep the element type (Float64: NaN propagates,
//     -0.0 < +0.0, as Julia's max / min);
//   * StatsBase.kurtosis of an integer or Float64 row is Float64 throughout:
//     m = mean(v) (Base.sum's pairwise Float64 sum, blocks of 1024 summed in
//     sequence, divided by n), then z = v[i] - m, z2 = z*z, cm2 += z2,
//     cm4 += z2*z2 in sequence, (cm4/n) / (cm2/n)^2 - 3.
// One lane per output, the reference's operations in the reference's order,
// so integer results are exact and Float64 results follow Julia's sequence
// (bar the @simd reassociation Julia may apply inside a 1024-element leaf).
// These are not the hot path (the products are Float32, which the kernels of
// kernels.hip / kurtosis.hip take): consecutive lanes take consecutive output
// groups, so each load instruction of a wave covers 64 groups' bytes.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include <cstdlib>
#include <limits>
#include <type_traits>

#include "bldp_impl.h"

// StatsBase rounds z*z before adding it (Julia contracts nothing without
// @fastmath / muladd); hipcc would otherwise fuse z2 = z*z; cm2 += z2 into fma.
#pragma clang fp contract(off)

namespace bldp {
namespace {

// Julia's Base.add_sum widening (the sum accumulator / result type)
template <typename T> struct SumT { typedef T type; };
template <> struct SumT<uint8_t> { typedef uint64_t type; };
template <> struct SumT<uint16_t> { typedef uint64_t type; };
template <> struct SumT<uint32_t> { typedef uint64_t type; };
template <> struct SumT<int8_t> { typedef int64_t type; };
template <> struct SumT<int16_t> { typedef int64_t type; };
template <> struct SumT<int32_t> { typedef int64_t type; };

template <typename T>
__device__ __forceinline__ T jmax(T a, T b) {
  if constexpr (sizeof(T) == 8 && (T)0.5 != 0) return __builtin_elementwise_maximum(a, b);
  else return a > b ? a : b;
}
template <typename T>
__device__ __forceinline__ T jmin(T a, T b) {
  if constexpr (sizeof(T) == 8 && (T)0.5 != 0) return __builtin_elementwise_minimum(a, b);
  else return a < b ? a : b;
}

// Base.mapreduce_impl (Base/reduce.jl) over n Float64 values v(0 .. n-1)
// with pairwise_blocksize 1024: halves [lo, mid], [mid+1, hi] with
// mid = lo + (hi - lo) >> 1 until a piece is no longer than 1024, which is
// summed in sequence from its first element.  Iterative, explicit stack.
template <typename V>
__device__ double jl_mapreduce_f64(int64_t n, const V &v) {
  if (n <= 0) return 0.0;
  if (n <= 1024) {  // one leaf (every fqavby of the BL products)
    double s = v(0);
    for (int64_t k = 1; k < n; ++k) s += v(k);
    return s;
  }
  int64_t lo[48], hi[48];
  double left[48];
  int state[48];
  int sp = 0;
  lo[0] = 0;
  hi[0] = n - 1;
  state[0] = 0;
  double val = 0.0;
  for (;;) {
    const int64_t L = lo[sp], H = hi[sp], M = L + ((H - L) >> 1);
    if (state[sp] == 0 && H - L < 1024) {
      double s = v(L);
      for (int64_t t = L + 1; t <= H; ++t) s += v(t);
      val = s;
    } else if (state[sp] == 0) {
      state[sp] = 1;
      ++sp;
      lo[sp] = L;
      hi[sp] = M;
      state[sp] = 0;
      continue;
    } else if (state[sp] == 1) {
      left[sp] = val;
      state[sp] = 2;
      ++sp;
      lo[sp] = M + 1;
      hi[sp] = H;
      state[sp] = 0;
      continue;
    } else {
      val = left[sp] + val;
    }
    if (sp == 0) break;
    --sp;
  }
  return val;
}

// sum(A; dims) of one slice as Base's reducedim takes it (_mapreducedim!):
// R = zero(Float64), R + mapreduce_impl(slice).  (Slices of <= 16 take the
// r = zero; r += A[i] loop instead: the same value, 0.0 + a1 = a1 but for
// a1 = -0.0, which the outer 0.0 + settles the same way.)
template <typename V>
__device__ double jl_dimsum_f64(int64_t n, const V &v) {
  return 0.0 + jl_mapreduce_f64(n, v);
}

template <typename TI, int OP>
__global__ __launch_bounds__(256) void k_reduce_typed(const TypedArgs a) {
  typedef typename SumT<TI>::type TS;
  // Float64 accumulation: Float64 sums, and every mean (Statistics.mean sums
  // the values converted to Float64: _mean_promote)
  constexpr bool F64ACC = OP == BLDP_OP_MEAN || (TI)0.5 != 0;
  const int64_t nout = a.nco * a.ni * a.nto * a.nbank;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < nout;
       e += (int64_t)gridDim.x * 256) {
    const int64_t co = e % a.nco;
    int64_t r = e / a.nco;
    const int64_t i = r % a.ni;
    r /= a.ni;
    const int64_t to = r % a.nto;
    const int64_t bank = r / a.nto;
    const TI *p = static_cast<const TI *>(a.in[bank]) + a.in_off + i * a.in_ld_i +
                  to * a.T * a.in_ld_t + co * a.F * a.in_cs;
    const int64_t oe = bank * a.out_bank + i * a.out_ld_i + to * a.out_ld_t + co;
    if constexpr (OP == BLDP_OP_MAX || OP == BLDP_OP_MIN) {
      TI acc = p[0];  // Julia seeds the reduction with the first element
      for (int64_t t = 0; t < a.T; ++t) {
        const TI *q = p + t * a.in_ld_t;
        for (int64_t k = (t == 0); k < a.F; ++k)
          acc = OP == BLDP_OP_MAX ? jmax<TI>(acc, q[k * a.in_cs]) : jmin<TI>(acc, q[k * a.in_cs]);
      }
      static_cast<TI *>(a.out)[oe] = acc;
    } else if constexpr (F64ACC) {
      // each spectrum's F channels as sum(reshape(A, (F, :, ...)); dims=1)
      // sums them (src/gbtworkerfunctions.jl:19), then the T spectral sums of
      // the time block the same way (time integration = fqav on axis 3)
      const int64_t F = a.F, cs = a.in_cs, ld = a.in_ld_t;
      const double s = jl_dimsum_f64(a.T, [&](int64_t t) {
        const TI *q = p + t * ld;
        return jl_dimsum_f64(F, [&](int64_t k) { return (double)q[k * cs]; });
      });
      if constexpr (OP == BLDP_OP_MEAN)
        static_cast<double *>(a.out)[oe] = s / (double)(a.F * a.T);
      else
        static_cast<double *>(a.out)[oe] = s;
    } else {  // integer sums: exact, wrapping like Julia's (U)Int64
      TS acc = 0;
      for (int64_t t = 0; t < a.T; ++t) {
        const TI *q = p + t * a.in_ld_t;
        for (int64_t k = 0; k < a.F; ++k) acc += (TS)q[k * a.in_cs];
      }
      static_cast<TS *>(a.out)[oe] = acc;
    }
  }
}

int64_t cdivt(int64_t x, int64_t y) { return (x + y - 1) / y; }
unsigned grid_for(int64_t n) { return (unsigned)std::min<int64_t>(cdivt(n, 256), 65536); }

// ---------------------------------------------------------------------------
// Coalesced form for the order-free reductions: integer sums (exact, wrapping:
// (U)Int64 addition is associative), max / min of integers and Float64 (NaN
// propagates and -0.0 < +0.0 whatever the order), and means of <= 32-bit
// integers whose partial sums stay below 2^53 (every order then gives the
// exact sum, which is what Julia's Float64 sum of the converted values is).
// The one-lane-per-group kernel above reads a group's F elements one at a
// time at a lane pitch of F elements; here each lane loads 16 contiguous bytes
// of a row (16 UInt8 SIGPROC samples, 8 UInt16, ...), so a wave-instruction
// reads 1 KiB contiguous, and the LPG lanes of a group combine by shuffle.
// A workgroup takes TPB consecutive time blocks of its 256 / LPG groups.
__device__ __forceinline__ uint32_t sad_u8(uint32_t x, uint32_t acc) {
  return __builtin_amdgcn_sad_u8(x, 0u, acc);  // acc + the 4 bytes of x
}
__device__ __forceinline__ uint32_t sad_u16(uint32_t x, uint32_t acc) {
  return __builtin_amdgcn_sad_u16(x, 0u, acc);  // acc + the 2 halfwords of x
}

template <typename TI, int OP>
struct Vec16 {
  // accumulator: exact integer sums in 64 bits (signed types biased to
  // unsigned and corrected at the end), max / min in the element type
  static constexpr bool SUM = OP == BLDP_OP_SUM || OP == BLDP_OP_MEAN;
  static constexpr int N = 16 / (int)sizeof(TI);  // elements per 16-byte load
  typedef typename std::conditional<SUM, uint64_t, TI>::type A;
  __device__ static A init() {
    // the identities of max / min (Float64: -Inf / +Inf, so an all -Inf group stays -Inf)
    typedef std::numeric_limits<TI> L;
    if constexpr (SUM) return 0;
    else if constexpr (OP == BLDP_OP_MAX) return L::has_infinity ? -L::infinity() : L::lowest();
    else return L::has_infinity ? L::infinity() : L::max();
  }
  __device__ static A add(A acc, uint4 q) {
    const uint32_t w[4] = {q.x, q.y, q.z, q.w};
    if constexpr (SUM && sizeof(TI) == 1) {
      const uint32_t b = std::is_signed<TI>::value ? 0x80808080u : 0u;
      uint32_t s = 0;
#pragma unroll
      for (int k = 0; k < 4; ++k) s = sad_u8(w[k] ^ b, s);
      return acc + s;
    } else if constexpr (SUM && sizeof(TI) == 2) {
      const uint32_t b = std::is_signed<TI>::value ? 0x80008000u : 0u;
      uint32_t s = 0;
#pragma unroll
      for (int k = 0; k < 4; ++k) s = sad_u16(w[k] ^ b, s);
      return acc + s;
    } else if constexpr (SUM && sizeof(TI) == 4) {
#pragma unroll
      for (int k = 0; k < 4; ++k) acc += (uint64_t)(int64_t)(TI)w[k];  // (sign-extended)
      return acc;
    } else if constexpr (SUM) {  // 64-bit: wrapping adds
      return acc + (((uint64_t)w[1] << 32) | w[0]) + (((uint64_t)w[3] << 32) | w[2]);
    } else {
      TI e[N];
      __builtin_memcpy(e, w, 16);
#pragma unroll
      for (int k = 0; k < N; ++k) acc = OP == BLDP_OP_MAX ? jmax<TI>(acc, e[k]) : jmin<TI>(acc, e[k]);
      return acc;
    }
  }
  __device__ static A combine(A x, A y) {
    if constexpr (SUM) return x + y;
    else return OP == BLDP_OP_MAX ? jmax<TI>(x, y) : jmin<TI>(x, y);
  }
  // one row's 16 bytes as a row accumulator R: 32 bits for 8- / 16-bit sums
  // (<= 16 rows of one lane stay below 2^24), else A
  typedef typename std::conditional<SUM && sizeof(TI) <= 2, uint32_t, A>::type R;
  __device__ static R row(uint4 q) {
    if constexpr (SUM && sizeof(TI) <= 2) return (R)add(0, q);
    else return add(init(), q);
  }
  __device__ static R rcombine(R x, R y) {
    if constexpr (SUM) return x + y;
    else return combine(x, y);
  }
  // the lanes' accumulators of a group -> the group's exact value
  __device__ static A shfl_xor(A x, int m) {
    if constexpr (sizeof(A) == 8) {
      uint64_t u;
      __builtin_memcpy(&u, &x, 8);
      const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)u, m, 64);
      const uint32_t hi = (uint32_t)__shfl_xor((int)(uint32_t)(u >> 32), m, 64);
      u = ((uint64_t)hi << 32) | lo;
      __builtin_memcpy(&x, &u, 8);
      return x;
    } else {
      return (A)__shfl_xor((int)x, m, 64);
    }
  }
};

typedef unsigned u4u __attribute__((ext_vector_type(4), aligned(4)));
__device__ __forceinline__ uint4 ld16(const char *p) {  // (dword-aligned: gfx950 dwordx4)
  const u4u v = __builtin_nontemporal_load(reinterpret_cast<const u4u *>(p));
  return make_uint4(v.x, v.y, v.z, v.w);
}

// One time block's result: the lanes' accumulators of a group folded, then
// stored by the group's first lane (signed 8- / 16-bit sums unbiased).
template <typename TI, int OP>
__device__ __forceinline__ void typed_vec_store(const TypedArgs &a, typename Vec16<TI, OP>::A acc,
                                                int lpg, bool st, int64_t bank, int64_t i,
                                                int64_t to, int64_t co) {
  typedef Vec16<TI, OP> V;
  typedef typename SumT<TI>::type TS;
  for (int m = 1; m < lpg; m <<= 1) acc = V::combine(acc, V::shfl_xor(acc, m));
  if (!st) return;
  const int64_t oe = bank * a.out_bank + i * a.out_ld_i + to * a.out_ld_t + co;
  if constexpr (V::SUM) {
    // undo the bias of signed 8- / 16-bit elements (x + 2^(bits-1) was summed)
    uint64_t u = acc;
    if constexpr (std::is_signed<TI>::value && sizeof(TI) <= 2)
      u -= (uint64_t)(a.F * a.T) << (8 * sizeof(TI) - 1);
    if constexpr (OP == BLDP_OP_MEAN) {
      const double sum = std::is_signed<TI>::value ? (double)(int64_t)u : (double)u;
      static_cast<double *>(a.out)[oe] = sum / (double)(a.F * a.T);
    } else {
      static_cast<TS *>(a.out)[oe] = (TS)u;
    }
  } else {
    static_cast<TI *>(a.out)[oe] = acc;
  }
}

// Grid: x = (column tile, time group) column tile fastest, y = IF, z = bank;
// a column tile is 256 / lpg groups (lpg lanes per group, k16 16-byte loads
// per lane per row), a time group tpb time blocks.
template <typename TI, int OP>
__global__ __launch_bounds__(256) void k_reduce_typed_vec(const TypedArgs a, int lpg, int k16,
                                                          int tpb, int64_t nct) {
  typedef Vec16<TI, OP> V;
  typedef typename V::A A;
  constexpr int NB = 16;  // 16-byte loads in flight per lane
  const int tid = threadIdx.x;
  const int64_t bx = blockIdx.x, ct = bx % nct, tg = bx / nct;
  const int64_t co = ct * (256 / lpg) + tid / lpg;  // this lane's group (lanes of a group: one wave)
  const int j = tid % lpg;
  const int64_t i = blockIdx.y;
  const int bank = blockIdx.z;
  const bool valid = co < a.nco;
  const int64_t T = a.T, ldb = a.in_ld_t * (int64_t)sizeof(TI), kb = 16 * (int64_t)lpg;
  const char *base = static_cast<const char *>(a.in[bank]) +
                     (a.in_off + i * a.in_ld_i + co * a.F) * (int64_t)sizeof(TI) + 16 * j;
  for (int b = 0; b < tpb; ++b) {
    const int64_t to = tg * tpb + b;
    if (to >= a.nto) break;  // (uniform over the workgroup)
    A acc = V::init();
    if (valid) {
      const char *p = base + to * T * ldb;
      if (k16 == 1) {
        for (int64_t r = 0; r < T; r += NB) {  // up to NB rows per batch, one wait each
          const int64_t n = T - r < NB ? T - r : NB;
          uint4 q[NB];
#pragma unroll
          for (int m = 0; m < NB; ++m)
            if (m < n) q[m] = ld16(p + (r + m) * ldb);
#pragma unroll
          for (int m = 0; m < NB; ++m)
            if (m < n) acc = V::add(acc, q[m]);
        }
      } else {
        for (int64_t r = 0; r < T; ++r, p += ldb) {
          int k = 0;
          for (; k + NB <= k16; k += NB) {
            uint4 q[NB];
#pragma unroll
            for (int m = 0; m < NB; ++m) q[m] = ld16(p + (k + m) * kb);
#pragma unroll
            for (int m = 0; m < NB; ++m) acc = V::add(acc, q[m]);
          }
          for (; k < k16; ++k) acc = V::add(acc, ld16(p + k * kb));
        }
      }
    }
    typed_vec_store<TI, OP>(a, acc, lpg, valid && j == 0, bank, i, to, co);
  }
}

// Short time blocks (T a power of two <= 16, one 16-byte load per lane per
// row): the rows of the workgroup's tpb blocks (tpb * T <= 16) are loaded in
// one batch, then folded into blocks, so a lane waits for memory once per
// workgroup instead of once per block.
template <typename TI, int OP, int NR>
__global__ __launch_bounds__(256) void k_reduce_typed_vec16(const TypedArgs a, int lpg, int tpb,
                                                            int64_t nct) {
  typedef Vec16<TI, OP> V;
  typedef typename V::R R;
  const int tid = threadIdx.x;
  const int64_t bx = blockIdx.x;
  const int64_t ct = bx % nct, tg = bx / nct;
  const int64_t co = ct * (256 / lpg) + tid / lpg;
  const int j = tid % lpg;
  const int64_t i = blockIdx.y;
  const int bank = blockIdx.z;
  const bool valid = co < a.nco;
  const int T = (int)a.T, tsh = __builtin_ctz((unsigned)T);
  const int64_t ldb = a.in_ld_t * (int64_t)sizeof(TI), to0 = tg * tpb;
  const int nb = (int)std::min<int64_t>(tpb, a.nto - to0), nrow = nb * T;
  R r[NR];
  if (valid) {
    const char *p = static_cast<const char *>(a.in[bank]) +
                    (a.in_off + i * a.in_ld_i + co * a.F) * (int64_t)sizeof(TI) + 16 * j +
                    to0 * T * ldb;
    uint4 q[NR];
#pragma unroll
    for (int m = 0; m < NR; ++m)
      if (m < nrow) q[m] = ld16(p + m * ldb);
#pragma unroll
    for (int m = 0; m < NR; ++m) r[m] = m < nrow ? V::row(q[m]) : V::row(make_uint4(0, 0, 0, 0));
  } else {
#pragma unroll
    for (int m = 0; m < NR; ++m) r[m] = R();
  }
  // rows -> time blocks: block b's value ends in r[b * T] (rows past nrow
  // are never folded into a stored block)
#pragma unroll
  for (int h = 1; h < NR; h *= 2)
    if (h < T) {
#pragma unroll
      for (int m = 0; m < NR; m += 2 * h) r[m] = V::rcombine(r[m], r[m + h]);
    }
#pragma unroll
  for (int m = 0; m < NR; ++m)
    if ((m & (T - 1)) == 0 && (m >> tsh) < nb)  // (uniform)
      typed_vec_store<TI, OP>(a, (typename V::A)r[m], lpg, valid && j == 0, bank, i,
                              to0 + (m >> tsh), co);
}

template <typename TI>
__global__ __launch_bounds__(256) void k_kurt_typed(const TypedArgs a, double *out) {
  const int64_t nrow = a.nco * a.ni * a.nbank;
  const int64_t n = a.nto;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < nrow;
       e += (int64_t)gridDim.x * 256) {
    const int64_t c = e % a.nco;
    const int64_t r = e / a.nco;
    const int64_t i = r % a.ni, bank = r / a.ni;
    const TI *p = static_cast<const TI *>(a.in[bank]) + a.in_off + i * a.in_ld_i + c * a.in_cs;
    // m = mean(v) = Base.sum(v) / n: mapreduce_impl over the whole row (no zero seed)
    const int64_t ld = a.in_ld_t;
    const double m = jl_mapreduce_f64(n, [&](int64_t t) { return (double)p[t * ld]; }) / (double)n;
    double cm2 = 0.0, cm4 = 0.0;
    for (int64_t t = 0; t < n; ++t) {
      const double z = (double)p[t * a.in_ld_t] - m;
      const double z2 = z * z;
      cm2 += z2;
      cm4 += z2 * z2;
    }
    cm4 /= (double)n;
    cm2 /= (double)n;
    out[e] = (cm4 / (cm2 * cm2)) - 3.0;
  }
}


// getkurtosis of 8- and 16-bit rows (SIGPROC nbits 8 / 16): k_kurt_typed's
// arithmetic with every lane on the 4 / 2 consecutive channels of one 32-bit
// word, so a wave-instruction reads 256 contiguous bytes instead of 64 / 128,
// and 16 spectra of loads in flight.  The mean's Float64 sum is exact for
// these types (|sum| < 2^53 for any n below 2^37), so the integer sum
// converted once is the value of Julia's pairwise Float64 sum; the moment
// loop runs in spectrum order per channel as StatsBase's does: bit-identical
// to k_kurt_typed (tests/test_gpu_typed.py).
template <typename TI>
__device__ __forceinline__ int32_t word_elem(uint32_t w, int k) {
  if constexpr (sizeof(TI) == 1)
    return std::is_signed<TI>::value ? (int32_t)(int8_t)(w >> (8 * k)) : (int32_t)((w >> (8 * k)) & 0xffu);
  else
    return std::is_signed<TI>::value ? (int32_t)(int16_t)(w >> (16 * k))
                                     : (int32_t)((w >> (16 * k)) & 0xffffu);
}
template <typename TI>
__global__ __launch_bounds__(256) void k_kurt_typed_w(const TypedArgs a, double *out) {
  constexpr int CPL = 4 / (int)sizeof(TI), U = 16;
  const int64_t ngl = a.nco / CPL, nrow = ngl * a.ni * a.nbank, n = a.nto;
  const int64_t ldb = a.in_ld_t * (int64_t)sizeof(TI);
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < nrow;
       e += (int64_t)gridDim.x * 256) {
    const int64_t q = e % ngl, r = e / ngl, i = r % a.ni, bank = r / a.ni;
    const char *p = static_cast<const char *>(a.in[bank]) +
                    (a.in_off + i * a.in_ld_i + q * CPL) * (int64_t)sizeof(TI);
    int64_t s[CPL];
#pragma unroll
    for (int k = 0; k < CPL; ++k) s[k] = 0;
    int64_t t = 0;
    for (; t + U <= n; t += U) {
      uint32_t w[U];
#pragma unroll
      for (int u = 0; u < U; ++u) w[u] = *reinterpret_cast<const uint32_t *>(p + (t + u) * ldb);
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int k = 0; k < CPL; ++k) s[k] += word_elem<TI>(w[u], k);
    }
    for (; t < n; ++t) {
      const uint32_t w = *reinterpret_cast<const uint32_t *>(p + t * ldb);
#pragma unroll
      for (int k = 0; k < CPL; ++k) s[k] += word_elem<TI>(w, k);
    }
    double m[CPL], cm2[CPL], cm4[CPL];
#pragma unroll
    for (int k = 0; k < CPL; ++k) {
      m[k] = (double)s[k] / (double)n;
      cm2[k] = 0.0;
      cm4[k] = 0.0;
    }
    t = 0;
    for (; t + U <= n; t += U) {
      uint32_t w[U];
#pragma unroll
      for (int u = 0; u < U; ++u) w[u] = *reinterpret_cast<const uint32_t *>(p + (t + u) * ldb);
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int k = 0; k < CPL; ++k) {
          const double z = (double)word_elem<TI>(w[u], k) - m[k];
          const double z2 = z * z;
          cm2[k] += z2;
          cm4[k] += z2 * z2;
        }
    }
    for (; t < n; ++t) {
      const uint32_t w = *reinterpret_cast<const uint32_t *>(p + t * ldb);
#pragma unroll
      for (int k = 0; k < CPL; ++k) {
        const double z = (double)word_elem<TI>(w, k) - m[k];
        const double z2 = z * z;
        cm2[k] += z2;
        cm4[k] += z2 * z2;
      }
    }
#pragma unroll
    for (int k = 0; k < CPL; ++k) {
      const double c4 = cm4[k] / (double)n, c2 = cm2[k] / (double)n;
      out[q * CPL + k + a.nco * r] = (c4 / (c2 * c2)) - 3.0;
    }
  }
}

// getkurtosis of 8-bit rows (SIGPROC nbits 8, the UInt8 products) from exact
// integer power sums.  For each channel the row's S1..S4 = sum of d^1..d^4,
// d = x - 128 (UInt8) or x (Int8), are integers that Int64 / UInt64 hold
// exactly (|d| <= 128, n <= 2^23), so any split of the time axis adds them
// back exactly: the window is read once by NW waves per tile of 64 lanes x W
// words (4 W channels a lane, W 32-bit words of each spectrum; 256 W
// contiguous bytes per wave-instruction), each wave summing a time slab, the
// slabs added in LDS (ds_add_u64), and, for long rows, time chunks of several workgroups added by
// k_kurt_int_final.  From the exact sums, with n the window's length:
// the central moments n cm2 = sum((x - mu)^2), n cm4 = sum((x - mu)^4) (which
// the shift leaves alone) re-centred exactly in Int64 and finished in Float64
// (kurt_from_sums), and kurtosis = (cm4 / n) / (cm2 / n)^2 - 3 as StatsBase's
// recipe defines it.  The recipe (src/gbtworkerfunctions.jl:197-202; Float64
// m, z, z^2, z^4 and sequential Float64 sums) differs from the exact ratio by
// its own rounding, at most (3 nt + 10) 2^-53 relative on k + 3; this path by
// at most ~150 2^-53 (tests hold the two to conftest.kurt_int_tol).  A row of
// one value gives NaN, as the recipe.
// 16-bit rows take the same plan and finish with wider sums (k_kurt_i16,
// below).  Plan option "typed_kurt": 1 (default) = these paths for 8- and
// 16-bit rows of dword-aligned words, 4- or 8-byte words a lane by
// kurt_int_plan's rule; 2 / 3 = 4- / 8-byte words (8: where the rows are
// 8-byte aligned); 0 = k_kurt_typed_w (the recipe's order, bit-exact).
struct KTM {
  int nw;           // waves per workgroup (time slabs)
  int wpl;          // words a lane (W: 1 or 2)
  int64_t ntile;    // tiles (64 lanes x W words) per row
  int64_t nchunk;   // time chunks (workgroups along time); 1: fused finish
  int64_t crow;     // spectra per chunk
  int64_t srow;     // spectra per wave slab (<= 1024: the lanes' 32-bit sums)
};
constexpr int64_t kI8MaxN = (int64_t)1 << 23;  // (the Int64 re-centring's bound)
// waves per CU one round of k_kurt_i8 / k_kurt_i16 should fill (k_kurt_i8:
// 58 VGPRs with 4-byte words, 8 waves a SIMD; 116 with 8-byte, 4 a SIMD;
// k_kurt_i16: 68 / 86); 12..32 are within ~5% of each other on the UInt8 and
// UInt16 0002 band and file (profiles/r06/kurtsweep_r06{j,m,w}.json)
constexpr int64_t kI8WavesPerCu = 16;
constexpr int64_t kI8MinSlab = 16;  // fewest spectra a wave's slab is cut to
constexpr int64_t kI8MaxSlab = 1024;  // most: |sum d^3| <= 2^21 x 1024 = 2^31 (Int32)

// The kurtosis of one channel from its exact sums S_k = sum of d^k (|d| <=
// 128, n <= 2^23).  Re-centred on c = the integer nearest the mean of d, in
// Int64 exactly (every term below 2^54):
//   T1 = S1 - n c, T2 = S2 - 2c S1 + n c^2, T3 = ..., T4 = ...  (binomial)
// then, with e = T1 / n (|e| <= 1/2),
//   n cm2 = T2 - T1 e,   n cm4 = T4 - 4e T3 + 6e^2 T2 - 3n e^4
// in Float64, and kurtosis = n (n cm4) / (n cm2)^2 - 3.  For integer data no
// value is nearer the mean than c is, so n e^4 <= n cm4 and n e^2 <= n cm2:
// each term above is at most 12 (T4), 20, 12 and 3 times n cm4, so the
// Float64 evaluation is within ~150 ulps of the exact ratio in the worst case
// (a few in practice); DESIGN.md §4 "Typed data".  A row of one value:
// T1 = T2 = T4 = 0 -> 0/0 = NaN, as the recipe.
__device__ __forceinline__ double kurt_from_sums(int64_t n, int64_t S1, uint64_t S2u, int64_t S3,
                                                 uint64_t S4u) {
  const int64_t S2 = (int64_t)S2u, S4 = (int64_t)S4u;
  const double dn = (double)n;
  const int32_t c = (int32_t)rint((double)S1 / dn);  // |c| <= 128
  const int64_t c2 = (int64_t)c * c, c3 = c2 * c, c4 = c2 * c2;
  const int64_t T1 = S1 - n * c;
  const int64_t T2 = S2 - 2 * c * S1 + n * c2;
  const int64_t T3 = S3 - 3 * c * S2 + 3 * c2 * S1 - n * c3;
  const int64_t T4 = S4 - 4 * c * S3 + 6 * c2 * S2 - 4 * c3 * S1 + n * c4;
  const double t1 = (double)T1, t2 = (double)T2, t3 = (double)T3, t4 = (double)T4;
  const double e = t1 / dn;
  const double m2 = t2 - t1 * e;
  const double m4 = t4 - e * (4.0 * t3 - e * (6.0 * t2 - 3.0 * t1 * e));
  return dn * m4 / (m2 * m2) - 3.0;
}

typedef short s2v __attribute__((ext_vector_type(2)));
typedef unsigned short u2v __attribute__((ext_vector_type(2)));

// 4 spectra x 4 channels of bytes (one word per spectrum) -> one word per
// channel holding its 4 spectra (v_perm_b32: 8 per 16 bytes)
__device__ __forceinline__ void transpose4(uint32_t w0, uint32_t w1, uint32_t w2, uint32_t w3,
                                           uint32_t (&T)[4]) {
  const uint32_t A = __builtin_amdgcn_perm(w1, w0, 0x05010400u);  // w0.b0 w1.b0 w0.b1 w1.b1
  const uint32_t B = __builtin_amdgcn_perm(w1, w0, 0x07030602u);  // w0.b2 w1.b2 w0.b3 w1.b3
  const uint32_t C = __builtin_amdgcn_perm(w3, w2, 0x05010400u);
  const uint32_t D = __builtin_amdgcn_perm(w3, w2, 0x07030602u);
  T[0] = __builtin_amdgcn_perm(C, A, 0x05040100u);
  T[1] = __builtin_amdgcn_perm(C, A, 0x07060302u);
  T[2] = __builtin_amdgcn_perm(D, B, 0x05040100u);
  T[3] = __builtin_amdgcn_perm(D, B, 0x07060302u);
}

// One batch of U spectra of a lane's W words (4 W channels), loaded: words
// past `cnt` are replaced by d = 0.  Sums of d = x - 128 (UInt8: the byte's
// top bit flipped, read as Int8) or x (Int8), |d| <= 128, per channel over 4
// spectra at a time: the words transposed so a word holds one channel's 4
// spectra, then
//   S1 += sdot4(T, 1), S2 += sdot4(T, T)                (<= 2^24 in 1024)
//   S3 += sdot2(d^2, d) over the Int16 halves           (|.| <= 2^31 in 1024)
//   S4 += udot2(d^2, d^2)                               (<= 2^31 per 8)
// (d^2 by v_pk_mul_lo_u16: <= 2^14), S4 moved to 64-bit sums per 8 spectra:
// ~4 VALU operations per byte.
template <bool SIGNED, int U, int W>
__device__ __forceinline__ void i8_batch(uint32_t (&w)[U][W], int cnt, int32_t (&s1)[4 * W],
                                         int32_t (&s2)[4 * W], int32_t (&s3)[4 * W],
                                         uint64_t (&s4)[4 * W]) {
  if (cnt < U) {  // (uniform: only a slab's last batch)
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int j = 0; j < W; ++j)
        if (u >= cnt) w[u][j] = SIGNED ? 0u : 0x80808080u;  // (d = 0: adds nothing)
  }
#pragma unroll
  for (int h = 0; h < U; h += 8) {
    uint32_t b4[4 * W];
#pragma unroll
    for (int k = 0; k < 4 * W; ++k) b4[k] = 0;
#pragma unroll
    for (int g = h; g < h + 8 && g < U; g += 4) {
      if (g >= cnt) break;  // (uniform: a short last batch)
#pragma unroll
      for (int j = 0; j < W; ++j) {
        uint32_t T[4];
        if (SIGNED)
          transpose4(w[g][j], w[g + 1][j], w[g + 2][j], w[g + 3][j], T);
        else
          transpose4(w[g][j] ^ 0x80808080u, w[g + 1][j] ^ 0x80808080u,
                     w[g + 2][j] ^ 0x80808080u, w[g + 3][j] ^ 0x80808080u, T);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int x = 4 * j + k;
          const int tk = (int)T[k];
          s1[x] = __builtin_amdgcn_sdot4(tk, 0x01010101, s1[x], false);
          s2[x] = __builtin_amdgcn_sdot4(tk, tk, s2[x], false);
          // Int16 halves: spectra (0, 2) and (1, 3), sign-extended
          const s2v e = __builtin_bit_cast(s2v, T[k] << 8) >> (short)8;
          const s2v o = __builtin_bit_cast(s2v, T[k]) >> (short)8;
          const u2v ue = __builtin_bit_cast(u2v, e), uo = __builtin_bit_cast(u2v, o);
          const u2v qe = ue * ue, qo = uo * uo;  // d^2 (mod 2^16: exact, <= 2^14)
          s3[x] = __builtin_amdgcn_sdot2(__builtin_bit_cast(s2v, qe), e, s3[x], false);
          s3[x] = __builtin_amdgcn_sdot2(__builtin_bit_cast(s2v, qo), o, s3[x], false);
          b4[x] = __builtin_amdgcn_udot2(qe, qe, b4[x], false);
          b4[x] = __builtin_amdgcn_udot2(qo, qo, b4[x], false);
        }
      }
    }
#pragma unroll
    for (int k = 0; k < 4 * W; ++k) s4[k] += b4[k];
  }
}

// Workgroup (tile, row, chunk): 64 lanes x W words (256 W channels) of one
// (bank x IF) row, NW waves on consecutive slabs of the chunk's spectra.  A
// wave streams its slab in batches of U spectra, the next batch's loads issued
// before the current one is summed (every load of a batch issued before the
// first is waited on: a short batch re-reads its last spectrum, in bounds, and
// the extra words become d = 0 by a select).
template <bool SIGNED, int W>
__global__ __launch_bounds__(1024) void k_kurt_i8(const TypedArgs a, const KTM m, double *out,
                                                  uint64_t *ws) {
  constexpr int U = 8;  // spectra of loads in flight per lane (and as many prefetched)
  constexpr int C = 4 * W;  // channels a lane
  typedef uint32_t wv_t __attribute__((ext_vector_type(W)));
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t ngl = a.nco / C, tile = blockIdx.x, r = blockIdx.y, chunk = blockIdx.z;
  const int64_t q = tile * 64 + lane;  // this lane's words
  const int64_t i = r % a.ni, bank = r / a.ni;
  const int64_t ct0 = chunk * m.crow, ct1 = min(a.nto, ct0 + m.crow);
  const int64_t t0 = min(ct1, ct0 + (int64_t)wave * m.srow), t1 = min(ct1, t0 + m.srow);
  int32_t s1[C], s2[C], s3[C];
  uint64_t s4[C];
#pragma unroll
  for (int k = 0; k < C; ++k) s1[k] = s2[k] = s3[k] = 0, s4[k] = 0;
  if (q < ngl && t1 > t0) {
    const int64_t ldb = a.in_ld_t;  // bytes (1-byte elements)
    // the tile's row start is uniform (a scalar base), the lane's words a
    // 32-bit offset: one address register for every load
    const char *base = static_cast<const char *>(a.in[bank]) + a.in_off + i * a.in_ld_i +
                       256 * W * tile;
    const uint32_t lofs = 4u * W * (uint32_t)lane;
    // spectra past the slab re-read its last one (in bounds; i8_batch drops
    // them), so no load sits behind a branch
    const int last = (int)(t1 - 1);  // (spectrum indices < 2^23: 32-bit, uniform)
    auto load = [&](uint32_t (&w)[U][W], int64_t t) {
      const int t32 = __builtin_amdgcn_readfirstlane((int)t);
#pragma unroll
      for (int u = 0; u < U; ++u) {
        // the row's byte offset held in scalar registers, so each load is
        // global_load_dword(x2) v, lofs, s[row] (no vector address arithmetic)
        const uint64_t ro = (uint64_t)((int64_t)min(t32 + u, last) * ldb);
        const uint64_t rs = ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(ro >> 32)) << 32) |
                            __builtin_amdgcn_readfirstlane((uint32_t)ro);
        const wv_t v = __builtin_nontemporal_load(reinterpret_cast<const wv_t *>(base + rs + lofs));
#pragma unroll
        for (int j = 0; j < W; ++j) w[u][j] = v[j];
      }
    };
    // two register buffers used in turn (no copies between them, so a
    // batch's sums wait only for its own loads)
    auto count = [&](int64_t t) { return (int)max((int64_t)0, min((int64_t)U, t1 - t)); };
    uint32_t wa[U][W], wb[U][W];
    int64_t t = t0;
    load(wa, t);
    for (;;) {
      const int ca = count(t), cb = count(t + U);
      load(wb, t + U);
      i8_batch<SIGNED, U, W>(wa, ca, s1, s2, s3, s4);
      if (cb == 0) break;
      load(wa, t + 2 * U);
      i8_batch<SIGNED, U, W>(wb, cb, s1, s2, s3, s4);
      if (count(t + 2 * U) == 0) break;
      t += 2 * U;
    }
  }
  // the slabs' sums added in LDS (two's complement: the signed sums too),
  // laid out [sum][channel of the lane][lane]: a wave's ds_add_u64 touches
  // 512 consecutive bytes
  __shared__ unsigned long long acc[4][C][64];
  for (int e = threadIdx.x; e < 4 * C * 64; e += blockDim.x) (&acc[0][0][0])[e] = 0ull;
  __syncthreads();
  if (q < ngl && t1 > t0) {
#pragma unroll
    for (int k = 0; k < C; ++k) {
      atomicAdd(&acc[0][k][lane], (unsigned long long)(int64_t)s1[k]);
      atomicAdd(&acc[1][k][lane], (unsigned long long)(int64_t)s2[k]);
      atomicAdd(&acc[2][k][lane], (unsigned long long)(int64_t)s3[k]);
      atomicAdd(&acc[3][k][lane], (unsigned long long)s4[k]);
    }
  }
  __syncthreads();
  for (int ch = threadIdx.x; ch < 64 * C; ch += blockDim.x) {
    const int64_t c = tile * 64 * C + ch;  // this workgroup's channels, coalesced
    const int l = ch / C, k = ch % C;  // (lane, channel of the lane)
    if (c < a.nco) {
      if (m.nchunk == 1) {
        out[c + a.nco * r] = kurt_from_sums(a.nto, (int64_t)acc[0][k][l], acc[1][k][l],
                                            (int64_t)acc[2][k][l], acc[3][k][l]);
      } else {
        const int64_t rows = a.ni * a.nbank;
#pragma unroll
        for (int s = 0; s < 4; ++s) ws[((chunk * 4 + s) * rows + r) * a.nco + c] = acc[s][k][l];
      }
    }
  }
}

// getkurtosis of 16-bit rows (SIGPROC nbits 16) the same way: d = x - 32768
// (UInt16) or x (Int16), |d| <= 2^15, and u = d + 32768 (the raw UInt16, or
// an Int16 with its top bit flipped), 0 <= u < 2^16.  Per channel, a lane's
// sums over a slab of <= 1024 spectra, every product one v_mad_u64_u32:
//   U1 += u (UInt32), U2 += u^2, U3 += d^2 u (UInt64; d^2 by v_mul_i32_i24),
//   S4 += d^2 d^2 (into a UInt64 per batch of 8 spectra, <= 2^63, then into a
//        96-bit sum: UInt64 + a UInt32 carry count),
// and at the slab's end, exactly in Int64 (m spectra, padding included: a
// padded spectrum has d = 0)
//   S1 = U1 - 2^15 m, S2 = U2 - 2^16 U1 + 2^30 m, S3 = U3 - 2^15 S2.
// The slabs and chunks add S3 and S4 as two limbs of radix 2^32 (each limb's
// sum fits 64 bits); kurt_from_limbs re-centres in Int128 (S4 <= 2^83) and
// finishes in Float64 as kurt_from_sums does, with the same bound.
__device__ __forceinline__ double i128_to_f64(__int128 v) {
  // correctly rounded: the top 64 bits with a sticky bit for the rest
  const bool neg = v < 0;
  const unsigned __int128 u = neg ? (unsigned __int128)0 - (unsigned __int128)v
                                  : (unsigned __int128)v;
  const uint64_t hi = (uint64_t)(u >> 64), lo = (uint64_t)u;
  double r;
  if (hi == 0) {
    r = (double)lo;
  } else {
    const int sh = 64 - __clzll((long long)hi);  // 1..64
    const uint64_t mask = sh >= 64 ? ~0ull : ((1ull << sh) - 1);
    const uint64_t top = (uint64_t)(u >> sh) | ((lo & mask) != 0);
    r = ldexp((double)top, sh);
  }
  return neg ? -r : r;
}

__device__ __forceinline__ double kurt_from_limbs(int64_t n, uint64_t L1, uint64_t L2,
                                                  uint64_t L3lo, uint64_t L3hi, uint64_t L4lo,
                                                  uint64_t L4hi) {
  typedef __int128 i128;
  const int64_t S1 = (int64_t)L1;
  const i128 S2 = (i128)L2;
  const i128 S3 = (i128)(int64_t)L3hi * ((i128)1 << 32) + (i128)L3lo;
  const i128 S4 = (i128)L4hi * ((i128)1 << 32) + (i128)L4lo;
  const double dn = (double)n;
  const int64_t c = (int64_t)rint((double)S1 / dn);  // |c| <= 2^15
  const i128 c1 = c, c2 = c1 * c1, c3 = c2 * c1, c4 = c2 * c2, nn = n;
  const i128 T1 = (i128)S1 - nn * c1;
  const i128 T2 = S2 - 2 * c1 * S1 + nn * c2;
  const i128 T3 = S3 - 3 * c1 * S2 + 3 * c2 * S1 - nn * c3;
  const i128 T4 = S4 - 4 * c1 * S3 + 6 * c2 * S2 - 4 * c3 * S1 + nn * c4;
  const double t1 = i128_to_f64(T1), t2 = i128_to_f64(T2), t3 = i128_to_f64(T3),
               t4 = i128_to_f64(T4);
  const double e = t1 / dn;
  const double m2 = t2 - t1 * e;
  const double m4 = t4 - e * (4.0 * t3 - e * (6.0 * t2 - 3.0 * t1 * e));
  return dn * m4 / (m2 * m2) - 3.0;
}

// Workgroup (tile, row, chunk): 64 lanes x W words (128 W channels) of one
// (bank x IF) row, NW waves on consecutive slabs; loads and batches as
// k_kurt_i8.
template <bool SIGNED, int W>
__global__ __launch_bounds__(1024) void k_kurt_i16(const TypedArgs a, const KTM m, double *out,
                                                   uint64_t *ws) {
  constexpr int U = 4;  // spectra of loads in flight per lane (and as many prefetched; 8: one
                        // UInt16 0002 file 13.6 vs 11.9 us, the band the same, 16: slower)
  constexpr int C = 2 * W;  // channels a lane
  typedef uint32_t wv_t __attribute__((ext_vector_type(W)));
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t ngl = a.nco / C, tile = blockIdx.x, r = blockIdx.y, chunk = blockIdx.z;
  const int64_t q = tile * 64 + lane;  // this lane's words
  const int64_t i = r % a.ni, bank = r / a.ni;
  const int64_t ct0 = chunk * m.crow, ct1 = min(a.nto, ct0 + m.crow);
  const int64_t t0 = min(ct1, ct0 + (int64_t)wave * m.srow), t1 = min(ct1, t0 + m.srow);
  uint32_t u1[C], s4c[C];
  uint64_t u2[C], u3[C], s4[C];
#pragma unroll
  for (int k = 0; k < C; ++k) u1[k] = 0, u2[k] = 0, u3[k] = 0, s4[k] = 0, s4c[k] = 0;
  int64_t m_rows = 0;  // spectra summed, padding included
  if (q < ngl && t1 > t0) {
    const int64_t ldb = 2 * a.in_ld_t;  // bytes
    const char *base = static_cast<const char *>(a.in[bank]) + 2 * (a.in_off + i * a.in_ld_i) +
                       256 * W * tile;
    const uint32_t lofs = 4u * W * (uint32_t)lane;
    const int last = (int)(t1 - 1);
    auto load = [&](uint32_t (&w)[U][W], int64_t t) {
      const int t32 = __builtin_amdgcn_readfirstlane((int)t);
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint64_t ro = (uint64_t)((int64_t)min(t32 + u, last) * ldb);
        const uint64_t rs = ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(ro >> 32)) << 32) |
                            __builtin_amdgcn_readfirstlane((uint32_t)ro);
        const wv_t v = __builtin_nontemporal_load(reinterpret_cast<const wv_t *>(base + rs + lofs));
#pragma unroll
        for (int j = 0; j < W; ++j) w[u][j] = v[j];
      }
    };
    auto batch = [&](uint32_t (&w)[U][W], int cnt) {
      if (cnt < U) {  // (uniform: only a slab's last batch)
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
          for (int j = 0; j < W; ++j)
            if (u >= cnt) w[u][j] = SIGNED ? 0u : 0x80008000u;  // (d = 0)
      }
      m_rows += U;
      uint64_t p4[C];
#pragma unroll
      for (int k = 0; k < C; ++k) p4[k] = 0;
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int j = 0; j < W; ++j) {
          const uint32_t x = SIGNED ? w[u][j] ^ 0x80008000u : w[u][j];  // two u
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const int k = 2 * j + h;
            const uint32_t uu = h ? x >> 16 : x & 0xffffu;
            const int32_t d = (int32_t)uu - 32768;
            const uint32_t dd = (uint32_t)(d * d);  // <= 2^30 (v_mul_i32_i24)
            u1[k] += uu;
            u2[k] += (uint64_t)uu * uu;
            u3[k] += (uint64_t)dd * uu;
            p4[k] += (uint64_t)dd * dd;
          }
        }
#pragma unroll
      for (int k = 0; k < C; ++k) {
        s4[k] += p4[k];
        s4c[k] += s4[k] < p4[k];  // (the carry out of the 64-bit sum)
      }
    };
    auto count = [&](int64_t t) { return (int)max((int64_t)0, min((int64_t)U, t1 - t)); };
    uint32_t wa[U][W], wb[U][W];
    int64_t t = t0;
    load(wa, t);
    for (;;) {
      const int ca = count(t), cb = count(t + U);
      load(wb, t + U);
      batch(wa, ca);
      if (cb == 0) break;
      load(wa, t + 2 * U);
      batch(wb, cb);
      if (count(t + 2 * U) == 0) break;
      t += 2 * U;
    }
  }
  // the slab's central sums (exact in Int64), added in LDS as 6 limbs (S1,
  // S2, S3 low / high 32 bits, S4 low / high 32 bits; the signed limbs in
  // two's complement)
  int64_t s1[C], s3[C];
  uint64_t s2[C];
#pragma unroll
  for (int k = 0; k < C; ++k) {
    s1[k] = (int64_t)u1[k] - ((int64_t)m_rows << 15);
    s2[k] = u2[k] - ((uint64_t)u1[k] << 16) + ((uint64_t)m_rows << 30);
    s3[k] = (int64_t)(u3[k] - (s2[k] << 15));
  }
  __shared__ unsigned long long acc[6][C][64];
  for (int e = threadIdx.x; e < 6 * C * 64; e += blockDim.x) (&acc[0][0][0])[e] = 0ull;
  __syncthreads();
  if (q < ngl && t1 > t0) {
#pragma unroll
    for (int k = 0; k < C; ++k) {
      atomicAdd(&acc[0][k][lane], (unsigned long long)s1[k]);
      atomicAdd(&acc[1][k][lane], (unsigned long long)s2[k]);
      atomicAdd(&acc[2][k][lane], (unsigned long long)(uint32_t)s3[k]);
      atomicAdd(&acc[3][k][lane], (unsigned long long)(s3[k] >> 32));
      atomicAdd(&acc[4][k][lane], (unsigned long long)(uint32_t)s4[k]);
      atomicAdd(&acc[5][k][lane], (unsigned long long)((s4[k] >> 32) + ((uint64_t)s4c[k] << 32)));
    }
  }
  __syncthreads();
  for (int ch = threadIdx.x; ch < 64 * C; ch += blockDim.x) {
    const int64_t c = tile * 64 * C + ch;  // this workgroup's channels, coalesced
    const int l = ch / C, k = ch % C;  // (lane, channel of the lane)
    if (c < a.nco) {
      if (m.nchunk == 1) {
        out[c + a.nco * r] = kurt_from_limbs(a.nto, acc[0][k][l], acc[1][k][l], acc[2][k][l],
                                             acc[3][k][l], acc[4][k][l], acc[5][k][l]);
      } else {
        const int64_t rows = a.ni * a.nbank;
#pragma unroll
        for (int s = 0; s < 6; ++s) ws[((chunk * 6 + s) * rows + r) * a.nco + c] = acc[s][k][l];
      }
    }
  }
}

// The chunks' sums of every channel added (exact: sums mod 2^64 in any
// order), then the kurtosis (nchunk > 1).  NS = 4 (k_kurt_i8: S1..S4) or 6
// (k_kurt_i16: S1, S2 and S3, S4 as two 32-bit-radix limbs).  Workgroup: 64
// consecutive channels x 16 waves, wave w adding chunks w, w + 16, ... (the
// 0001 product: 512 channels of 100+ chunks -- one thread a channel walking
// the chunks in turn paid a dependent load per chunk, ~0.26 us each).
template <int NS>
__global__ __launch_bounds__(1024) void k_kurt_int_final(const TypedArgs a, const KTM m,
                                                         double *out, const uint64_t *ws) {
  const int64_t rows = a.ni * a.nbank, n = a.nco * rows;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t e = (int64_t)blockIdx.x * 64 + lane;
  uint64_t S[NS];
#pragma unroll
  for (int s = 0; s < NS; ++s) S[s] = 0;
  if (e < n)
    for (int64_t c = wave; c < m.nchunk; c += 16)
#pragma unroll
      for (int s = 0; s < NS; ++s) S[s] += ws[(c * NS + s) * n + e];
  __shared__ unsigned long long acc[NS][64];
  if (threadIdx.x < NS * 64) (&acc[0][0])[threadIdx.x] = 0ull;
  __syncthreads();
#pragma unroll
  for (int s = 0; s < NS; ++s) atomicAdd(&acc[s][lane], (unsigned long long)S[s]);
  __syncthreads();
  if (wave == 0 && e < n) {
    if constexpr (NS == 4)
      out[e] = kurt_from_sums(a.nto, (int64_t)acc[0][lane], acc[1][lane], (int64_t)acc[2][lane],
                              acc[3][lane]);
    else
      out[e] = kurt_from_limbs(a.nto, acc[0][lane], acc[1][lane], acc[2][lane], acc[3][lane],
                               acc[4][lane], acc[5][lane]);
  }
}

// The k_kurt_i8 / k_kurt_i16 geometry, or false when the path does not
// apply.
bool kurt_int_plan(const TypedArgs &a, KTM *m) {
  const int64_t es = (int64_t)dtype_size(a.dtype), cpw = 4 / std::max<int64_t>(1, es);
  if ((es != 1 && es != 2) || !opt(OPT_TYPED_KURT)) return false;
  if (a.in_cs != 1 || a.nco % cpw || a.nto < 1 || a.nto > kI8MaxN) return false;
  // (byte offsets of the window and its rows)
  const int64_t off = a.in_off * es, ldi = a.in_ld_i * es, ldt = a.in_ld_t * es;
  if (off % 4 || (a.ni > 1 && ldi % 4) || (a.nto > 1 && ldt % 4)) return false;
  for (int b = 0; b < a.nbank; ++b)
    if ((uintptr_t)a.in[b] % 4) return false;
  const int64_t rows = a.ni * a.nbank;
  // (probe knobs, read once: BLDP_KURT_I8_WAVES_PER_CU 4..64, BLDP_KURT_I8_MIN_SLAB 8..4096)
  static const int64_t per_cu = [] {
    const char *e = getenv("BLDP_KURT_I8_WAVES_PER_CU");
    return e ? std::min<int64_t>(64, std::max<int64_t>(4, atoi(e))) : kI8WavesPerCu;
  }();
  static const int64_t min_slab = [] {
    const char *e = getenv("BLDP_KURT_I8_MIN_SLAB");
    return e ? std::min<int64_t>(4096, std::max<int64_t>(8, atoi(e))) : kI8MinSlab;
  }();
  const int64_t want = per_cu * (int64_t)std::max(1, a.num_cus);
  // 8-byte loads (2 words a lane: 512 contiguous bytes a wave-load) where
  // every row start is 8-byte aligned and the tiles alone, cut into slabs,
  // fill the round (the UInt8 0002 band: 1024 tiles, 30.8 vs 33.4 us); 4-byte
  // loads otherwise (one UInt8 0002 file: 128 tiles of 8 channels a lane,
  // 12.1 vs 8.6 us; profiles/r06/kurtsweep_r06m.json)
  bool w2a = a.nco % (2 * cpw) == 0 && off % 8 == 0 && (a.ni == 1 || ldi % 8 == 0) &&
             (a.nto == 1 || ldt % 8 == 0);
  for (int b = 0; w2a && b < a.nbank; ++b) w2a = (uintptr_t)a.in[b] % 8 == 0;
  const bool w2 = w2a && cdivt(a.nco / (2 * cpw), 64) * rows *
                                 std::min<int64_t>(16, cdivt(a.nto, min_slab)) >= want;
  const int64_t form = opt(OPT_TYPED_KURT);  // 1: by the rule, 2: 4-byte, 3: 8-byte words
  m->wpl = (form == 1 && w2) || (form == 3 && w2a) ? 2 : 1;
  m->ntile = cdivt(a.nco / (cpw * m->wpl), 64);
  // waves for one round of kI8WavesPerCu: NW waves a tile (<= 16,
  // never slabs under 16 spectra), then time chunks while the tiles still
  // leave the CUs short (0001: 512 channels = 2 tiles a row, ~10^6 spectra),
  // and never slabs over 1024 (the lanes' 32-bit sums).  The UInt8 0002
  // band: 1024 tiles x 4 waves of 70 spectra; one UInt8 0002 file: 256 tiles
  // x 16 waves of 18
  const int64_t tiles = m->ntile * rows;
  m->nw = (int)std::max<int64_t>(1, std::min<int64_t>({16, cdivt(want, tiles),
                                                       cdivt(a.nto, min_slab)}));
  const int64_t waves = tiles * m->nw;
  int64_t nchunk = std::max<int64_t>(1, std::min(cdivt(want, waves),
                                                 a.nto / (min_slab * (int64_t)m->nw)));
  nchunk = std::max(nchunk, cdivt(a.nto, (int64_t)m->nw * kI8MaxSlab));
  m->crow = cdivt(a.nto, nchunk);
  m->srow = cdivt(m->crow, m->nw);
  m->crow = m->srow * m->nw;
  m->nchunk = cdivt(a.nto, m->crow);
  return m->ntile <= INT32_MAX && rows <= 65535 && m->nchunk <= 65535;
}

// Scratch for a chunked plan's partial sums: NS UInt64 a channel a chunk.
size_t kurt_int_ws_bytes(const TypedArgs &a, const KTM &m) {
  const size_t ns = dtype_size(a.dtype) == 1 ? 4 : 6;  // sums a channel
  return (size_t)m.nchunk * ns * (size_t)(a.ni * a.nbank * a.nco) * sizeof(uint64_t);
}

// The coalesced kernel's geometry for this window, or false when it does not
// apply (Float64 sums, 64-bit means and inexact 32-bit means keep the
// reference's order on k_reduce_typed; windows without dword-aligned 16-byte
// rows of whole groups, too).
// Dynamic LDS per k_reduce_typed_vec16 workgroup as a cap on the workgroups
// resident per CU (as kIlShm in kernels.hip); 0 = no cap: 2 / 3 / 4 per CU
// lost 8-85% on the UInt8 / UInt16 0002 band and file (round 5,
// profiles/r05/ab_typed_r05g2.json).  (Round 5: a
// persistent, software-pipelined form -- tiles walked by 1..4 workgroups per
// CU, the next tile's loads issued before the current one's folds -- was
// slower on the UInt8 0002 band at every width: 72 / 43 / 32 vs 29 us,
// profiles/r05/typed_pipe_r05d.json; removed.)
constexpr unsigned kTypedShm = 0;

struct TVec {
  int lpg, k16, tpb;
  int nr;  // k_reduce_typed_vec16's rows per batch (4), 0: k_reduce_typed_vec
  int64_t nct, grid_x;
};
bool typed_vec_plan(const TypedArgs &a, int op, int num_cus, TVec *v) {
  const int64_t sz = (int64_t)dtype_size(a.dtype);
  const bool f64 = a.dtype == BLDP_DT_F64;
  if (f64 && (op == BLDP_OP_SUM || op == BLDP_OP_MEAN)) return false;
  if (op == BLDP_OP_MEAN && (sz == 8 || (sz == 4 && a.F * a.T > (1 << 21)))) return false;
  if (a.in_cs != 1 || (a.F * sz) % 16 != 0 || a.ni > 65535 || a.nbank > 65535) return false;
  // every 16-byte load on a dword boundary
  auto al = [](int64_t bytes) { return bytes % 4 == 0; };
  for (int b = 0; b < a.nbank; ++b)
    if ((uintptr_t)a.in[b] % 4) return false;
  if (!al(a.in_off * sz) || (a.ni > 1 && !al(a.in_ld_i * sz)) ||
      (a.nto * a.T > 1 && !al(a.in_ld_t * sz)))
    return false;
  const int64_t g16 = a.F * sz / 16;
  int lpg = 1;
  while (lpg < 64 && g16 % (2 * lpg) == 0) lpg *= 2;
  v->lpg = lpg;
  v->k16 = (int)(g16 / lpg);
  v->nct = cdivt(a.nco, 256 / lpg);
  // time blocks per workgroup: up to 4 rows where the blocks are short,
  // halved while the grid holds fewer than 8 workgroups per CU; one batch of
  // 4 rows.  4 rows (20 VGPRs, every wave resident) beat 8 and 16 (37 / 68
  // VGPRs) on the 8-bit 0002 file and band (profiles/r04/typed_rows_r04e.json;
  // the 8- and 16-row forms and their option typed_rows removed in round 5)
  constexpr int64_t rows = 4;
  const bool batch = v->k16 == 1 && a.T <= rows && (a.T & (a.T - 1)) == 0;
  int64_t tpb = std::max<int64_t>(1, std::min<int64_t>(a.nto, (batch ? rows : 16) /
                                                                  std::max<int64_t>(1, a.T)));
  while (tpb > 1 && v->nct * cdivt(a.nto, tpb) * a.ni * a.nbank < (int64_t)8 * num_cus) tpb /= 2;
  v->tpb = (int)tpb;
  v->nr = 0;
  if (batch) {
    v->nr = 4;  // (tpb * T <= 4)
  }
  v->grid_x = v->nct * cdivt(a.nto, tpb);
  return v->grid_x <= INT32_MAX;
}

template <typename TI>
hipError_t launch_typed_vec(const TypedArgs &a, int op, const TVec &v, hipStream_t s) {
  const dim3 g((unsigned)v.grid_x, (unsigned)a.ni, (unsigned)a.nbank), b(256);
  switch (op) {
#define BLDP_TV(O)                                                                            \
  if (v.nr == 4)                                                                              \
    hipLaunchKernelGGL((k_reduce_typed_vec16<TI, O, 4>), g, b, kTypedShm, s, a, v.lpg, v.tpb,  \
                       v.nct);                                                                \
  else                                                                                        \
    hipLaunchKernelGGL((k_reduce_typed_vec<TI, O>), g, b, 0, s, a, v.lpg, v.k16, v.tpb, v.nct); \
  break;
    case BLDP_OP_SUM:
      if constexpr (!std::is_floating_point<TI>::value) { BLDP_TV(BLDP_OP_SUM) }
      return hipErrorInvalidValue;
    case BLDP_OP_MEAN:
      if constexpr (!std::is_floating_point<TI>::value && sizeof(TI) <= 4) { BLDP_TV(BLDP_OP_MEAN) }
      return hipErrorInvalidValue;
    case BLDP_OP_MAX: BLDP_TV(BLDP_OP_MAX)
    case BLDP_OP_MIN: BLDP_TV(BLDP_OP_MIN)
#undef BLDP_TV
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

template <typename TI>
hipError_t launch_typed_op(const TypedArgs &a, int op, hipStream_t s) {
  TVec v;
  if (opt(OPT_TYPED_VEC) && typed_vec_plan(a, op, a.num_cus, &v))
    return launch_typed_vec<TI>(a, op, v, s);
  const int64_t n = a.nco * a.ni * a.nto * a.nbank;
  const dim3 g(grid_for(n)), b(256);
  switch (op) {
    case BLDP_OP_SUM: hipLaunchKernelGGL((k_reduce_typed<TI, BLDP_OP_SUM>), g, b, 0, s, a); break;
    case BLDP_OP_MEAN: hipLaunchKernelGGL((k_reduce_typed<TI, BLDP_OP_MEAN>), g, b, 0, s, a); break;
    case BLDP_OP_MAX: hipLaunchKernelGGL((k_reduce_typed<TI, BLDP_OP_MAX>), g, b, 0, s, a); break;
    case BLDP_OP_MIN: hipLaunchKernelGGL((k_reduce_typed<TI, BLDP_OP_MIN>), g, b, 0, s, a); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

template <typename TI>
hipError_t launch_kurt_t(const TypedArgs &a, double *out, hipStream_t s) {
  const int64_t n = a.nco * a.ni * a.nbank;
  if constexpr (sizeof(TI) <= 2 && std::is_integral<TI>::value) {
    // exact integer moments (k_kurt_i8 / k_kurt_i16)
    KTM m;
    // (chunked: only into scratch the caller sized for this same plan)
    if (kurt_int_plan(a, &m) &&
        (m.nchunk == 1 || (a.ws && kurt_int_ws_bytes(a, m) <= a.ws_bytes))) {
      const dim3 g((unsigned)m.ntile, (unsigned)(a.ni * a.nbank), (unsigned)m.nchunk);
      uint64_t *ws = static_cast<uint64_t *>(a.ws);
      constexpr bool sg = std::is_signed<TI>::value;
      constexpr int ns = sizeof(TI) == 1 ? 4 : 6;
      if constexpr (sizeof(TI) == 1) {
        if (m.wpl == 2)
          hipLaunchKernelGGL((k_kurt_i8<sg, 2>), g, dim3(64 * m.nw), 0, s, a, m, out, ws);
        else
          hipLaunchKernelGGL((k_kurt_i8<sg, 1>), g, dim3(64 * m.nw), 0, s, a, m, out, ws);
      } else {
        if (m.wpl == 2)
          hipLaunchKernelGGL((k_kurt_i16<sg, 2>), g, dim3(64 * m.nw), 0, s, a, m, out, ws);
        else
          hipLaunchKernelGGL((k_kurt_i16<sg, 1>), g, dim3(64 * m.nw), 0, s, a, m, out, ws);
      }
      if (m.nchunk > 1)
        hipLaunchKernelGGL(k_kurt_int_final<ns>, dim3((unsigned)cdivt(n, 64)), dim3(1024), 0, s,
                           a, m, out, ws);
      return hipGetLastError();
    }
  }
  if constexpr (sizeof(TI) <= 2) {  // 32-bit words of 4 / 2 channels (k_kurt_typed_w)
    constexpr int64_t cpl = 4 / (int64_t)sizeof(TI);
    bool ok = opt(OPT_TYPED_VEC) && a.in_cs == 1 && a.nco % cpl == 0 && a.nto > 0 &&
              (a.in_off * (int64_t)sizeof(TI)) % 4 == 0 &&
              (a.ni == 1 || (a.in_ld_i * (int64_t)sizeof(TI)) % 4 == 0) &&
              (a.in_ld_t * (int64_t)sizeof(TI)) % 4 == 0;
    for (int b = 0; ok && b < a.nbank; ++b) ok = (uintptr_t)a.in[b] % 4 == 0;
    if (ok) {
      hipLaunchKernelGGL((k_kurt_typed_w<TI>), dim3(grid_for(n / cpl)), dim3(256), 0, s, a, out);
      return hipGetLastError();
    }
  }
  hipLaunchKernelGGL((k_kurt_typed<TI>), dim3(grid_for(n)), dim3(256), 0, s, a, out);
  return hipGetLastError();
}

}  // namespace

size_t kurtosis_typed_ws_bytes(const TypedArgs &a) {
  KTM m;
  if (!kurt_int_plan(a, &m) || m.nchunk == 1) return 0;
  return kurt_int_ws_bytes(a, m);
}

size_t dtype_size(int dtype) {
  switch (dtype) {
    case BLDP_DT_F32: case BLDP_DT_U32: case BLDP_DT_I32: return 4;
    case BLDP_DT_F64: case BLDP_DT_U64: case BLDP_DT_I64: return 8;
    case BLDP_DT_U16: case BLDP_DT_I16: return 2;
    case BLDP_DT_U8: case BLDP_DT_I8: return 1;
  }
  return 0;
}

int typed_out_dtype(int dtype, int op) {
  if (!dtype_size(dtype) || op < BLDP_OP_SUM || op > BLDP_OP_MIN) return -1;
  if (op == BLDP_OP_MAX || op == BLDP_OP_MIN) return dtype;
  if (dtype == BLDP_DT_F32) return BLDP_DT_F32;
  if (op == BLDP_OP_MEAN) return BLDP_DT_F64;
  switch (dtype) {
    case BLDP_DT_U8: case BLDP_DT_U16: case BLDP_DT_U32: case BLDP_DT_U64: return BLDP_DT_U64;
    case BLDP_DT_I8: case BLDP_DT_I16: case BLDP_DT_I32: case BLDP_DT_I64: return BLDP_DT_I64;
  }
  return BLDP_DT_F64;
}

hipError_t launch_reduce_typed(const TypedArgs &a, int op, hipStream_t s) {
  if (a.nco * a.ni * a.nto == 0) return hipSuccess;
  switch (a.dtype) {
    case BLDP_DT_F64: return launch_typed_op<double>(a, op, s);
    case BLDP_DT_U8: return launch_typed_op<uint8_t>(a, op, s);
    case BLDP_DT_U16: return launch_typed_op<uint16_t>(a, op, s);
    case BLDP_DT_U32: return launch_typed_op<uint32_t>(a, op, s);
    case BLDP_DT_U64: return launch_typed_op<uint64_t>(a, op, s);
    case BLDP_DT_I8: return launch_typed_op<int8_t>(a, op, s);
    case BLDP_DT_I16: return launch_typed_op<int16_t>(a, op, s);
    case BLDP_DT_I32: return launch_typed_op<int32_t>(a, op, s);
    case BLDP_DT_I64: return launch_typed_op<int64_t>(a, op, s);
  }
  return hipErrorInvalidValue;
}

hipError_t launch_kurtosis_typed(const TypedArgs &a, double *out, hipStream_t s) {
  if (a.nco * a.ni == 0) return hipSuccess;
  switch (a.dtype) {
    case BLDP_DT_F64: return launch_kurt_t<double>(a, out, s);
    case BLDP_DT_U8: return launch_kurt_t<uint8_t>(a, out, s);
    case BLDP_DT_U16: return launch_kurt_t<uint16_t>(a, out, s);
    case BLDP_DT_U32: return launch_kurt_t<uint32_t>(a, out, s);
    case BLDP_DT_U64: return launch_kurt_t<uint64_t>(a, out, s);
    case BLDP_DT_I8: return launch_kurt_t<int8_t>(a, out, s);
    case BLDP_DT_I16: return launch_kurt_t<int16_t>(a, out, s);
    case BLDP_DT_I32: return launch_kurt_t<int32_t>(a, out, s);
    case BLDP_DT_I64: return launch_kurt_t<int64_t>(a, out, s);
  }
  return hipErrorInvalidValue;
}

}  // namespace bldp
