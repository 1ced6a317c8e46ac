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

int64_t cdivt(int64_t x, int64_t y) { return (x + y - 1) / y; }
unsigned grid_for(int64_t n) { return (unsigned)std::min<int64_t>(cdivt(n, 256), 65536); }

template <typename TI>
hipError_t launch_typed_op(const TypedArgs &a, int op, hipStream_t s) {
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
  hipLaunchKernelGGL((k_kurt_typed<TI>), dim3(grid_for(n)), dim3(256), 0, s, a, out);
  return hipGetLastError();
}

}  // namespace

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
