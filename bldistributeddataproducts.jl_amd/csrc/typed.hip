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
//     Float64 stay as they are), so every sum here is exact (wrapping like
//     Julia's Int64 / UInt64 on overflow) or a Float64 sum taken in the
//     reference's order (the n channels in sequence, spectrum after spectrum);
//   * mean(...; dims = 1) is Float64 for integer and Float64 input: the sum of
//     the values converted to Float64, divided by n (for integers the exact sum
//     converted once, which is the same number while it stays below 2^53);
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

template <typename TI, int OP>
__global__ __launch_bounds__(256) void k_reduce_typed(const TypedArgs a) {
  typedef typename SumT<TI>::type TS;
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
    } else {
      TS acc = 0;
      for (int64_t t = 0; t < a.T; ++t) {
        const TI *q = p + t * a.in_ld_t;
        for (int64_t k = 0; k < a.F; ++k) acc += (TS)q[k * a.in_cs];
      }
      if constexpr (OP == BLDP_OP_MEAN)
        static_cast<double *>(a.out)[oe] = (double)acc / (double)(a.F * a.T);
      else
        static_cast<TS *>(a.out)[oe] = acc;
    }
  }
}

// Base.sum of a Float64 row (the values converted to Float64): mapreduce_impl
// with pairwise_blocksize 1024 — halves [lo, mid], [mid+1, hi] with
// mid = lo + (hi - lo) >> 1 until a piece is shorter than 1024 + 1, which is
// summed in sequence from its first element.  Iterative, explicit stack.
template <typename TI>
__device__ double jl_pairwise_f64(const TI *p, int64_t ld, int64_t n) {
  if (n <= 0) return 0.0;
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
      double v = (double)p[L * ld];
      for (int64_t t = L + 1; t <= H; ++t) v += (double)p[t * ld];
      val = v;
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
    const double m = jl_pairwise_f64<TI>(p, a.in_ld_t, n) / (double)n;
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
