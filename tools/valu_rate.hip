// valu_rate.hip — issue rate of the VALU instructions the 8-bit kurtosis
// kernel (typed.hip k_kurt_i8) and its alternatives are built from, on one
// MI355X: each kernel runs 8 independent chains of one operation per lane
// (one VALU instruction per step by inline asm, so no chain folds), every SIMD full (grid of 8 waves per SIMD), and reports
// cycles per wave-instruction per SIMD = wall x clock x SIMDs / wave-instructions.
//
//   hipcc --offload-arch=gfx950 -O3 -o build/valu_rate tools/valu_rate.hip
//   ./build/valu_rate            (JSON lines)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef short s2v __attribute__((ext_vector_type(2)));
typedef unsigned short u2v __attribute__((ext_vector_type(2)));

#define CK(x)                                                                    \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) {                                                      \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                   \
    }                                                                            \
  } while (0)

constexpr int kIters = 4096, kChains = 8;

template <int OP>
__global__ __launch_bounds__(256) void k_rate(const unsigned *in, unsigned *out) {
  unsigned a[kChains];
  uint64_t b[kChains];
  const unsigned x = in[threadIdx.x & 63], y = in[64 + (threadIdx.x & 63)];
#pragma unroll
  for (int c = 0; c < kChains; ++c) {
    a[c] = x + c;
    b[c] = (uint64_t)y << c;
  }
  for (int it = 0; it < kIters; ++it) {
#pragma unroll
    for (int c = 0; c < kChains; ++c) {
      // one instruction each (VALU only), so nothing folds the chain
      if constexpr (OP == 0) asm volatile("v_dot4c_i32_i8 %0, %0, %1" : "+v"(a[c]) : "v"(y));
      if constexpr (OP == 1) asm volatile("v_dot2c_i32_i16 %0, %0, %1" : "+v"(a[c]) : "v"(y));
      if constexpr (OP == 2) asm volatile("v_dot2_u32_u16 %0, %0, %1, %0" : "+v"(a[c]) : "v"(y));
      if constexpr (OP == 3) asm volatile("v_pk_mul_lo_u16 %0, %0, %1" : "+v"(a[c]) : "v"(y));
      if constexpr (OP == 4) asm volatile("v_perm_b32 %0, %0, %1, %1" : "+v"(a[c]) : "v"(y));
      if constexpr (OP == 5) asm volatile("v_pk_ashrrev_i16 %0, 3, %0" : "+v"(a[c]));
      if constexpr (OP == 6) asm volatile("v_mad_u32_u24 %0, %0, %1, %0" : "+v"(a[c]) : "v"(y));
      if constexpr (OP == 7) asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[c]) : "v"(y));
      if constexpr (OP == 8) asm volatile("v_lshl_add_u64 %0, %0, 0, %0" : "+v"(b[c]));
      if constexpr (OP == 9) asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(b[c]) : "v"(a[c]), "v"(y) : "vcc");
      if constexpr (OP == 10) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(a[c]) : "v"(y));
      if constexpr (OP == 11) asm volatile("v_fma_f64 %0, %0, %0, %0" : "+v"(b[c]));
      if constexpr (OP == 12) asm volatile("v_add_f64 %0, %0, %0" : "+v"(b[c]));
      if constexpr (OP == 13) asm volatile("v_cvt_f64_f32 %0, %1" : "=v"(b[c]) : "v"(a[c]));
      if constexpr (OP == 14) asm volatile("v_fma_f32 %0, %0, %1, %0" : "+v"(a[c]) : "v"(y));
      if constexpr (OP == 15) asm volatile("v_pk_add_u16 %0, %0, %1" : "+v"(a[c]) : "v"(y));
      if constexpr (OP == 16) asm volatile("v_and_b32 %0, %0, %1" : "+v"(a[c]) : "v"(y));
      if constexpr (OP == 17) asm volatile("v_bfe_u32 %0, %0, 8, 8" : "+v"(a[c]));
      if constexpr (OP == 18) asm volatile("v_mul_i32_i24 %0, %0, %1" : "+v"(a[c]) : "v"(y));
      if constexpr (OP == 19) asm volatile("v_mad_i64_i32 %0, vcc, %1, %2, %0" : "+v"(b[c]) : "v"(a[c]), "v"(y) : "vcc");
      if constexpr (OP == 20) asm volatile("v_pk_mad_u16 %0, %0, %1, %0" : "+v"(a[c]) : "v"(y));
      if constexpr (OP == 21) asm volatile("v_sad_u8 %0, %0, %1, %0" : "+v"(a[c]) : "v"(y));
      if constexpr (OP == 22) asm volatile("v_lshrrev_b32 %0, 8, %0" : "+v"(a[c]));
    }
  }
  unsigned s = 0;
#pragma unroll
  for (int c = 0; c < kChains; ++c) s += a[c] + (unsigned)b[c] + (unsigned)(b[c] >> 32);
  if (s == 0x12345678u) out[threadIdx.x] = s;
}

static const char *kName[] = {"v_dot4c_i32_i8",  "v_dot2c_i32_i16", "v_dot2_u32_u16", "v_pk_mul_lo_u16",
                              "v_perm_b32",      "v_pk_ashrrev_i16", "v_mad_u32_u24", "v_add_u32",
                              "v_lshl_add_u64", "v_mad_u64_u32", "v_mul_lo_u32", "v_fma_f64",
                              "v_add_f64", "v_cvt_f64_f32", "v_fma_f32", "v_pk_add_u16",
                              "v_and_b32", "v_bfe_u32", "v_mul_i32_i24", "v_mad_i64_i32",
                              "v_pk_mad_u16", "v_sad_u8", "v_lshrrev_b32"};

template <int OP>
void run(const unsigned *in, unsigned *out, int ncu, int clock_khz) {
  const int grid = ncu * 8;  // 8 waves per SIMD of 256-thread workgroups: 2 wave-slots each
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  hipLaunchKernelGGL(k_rate<OP>, dim3(grid), dim3(256), 0, 0, in, out);
  CK(hipDeviceSynchronize());
  float best = 1e30f;
  for (int r = 0; r < 5; ++r) {
    CK(hipEventRecord(e0, 0));
    hipLaunchKernelGGL(k_rate<OP>, dim3(grid), dim3(256), 0, 0, in, out);
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    best = ms < best ? ms : best;
  }
  const double winst = (double)grid * 4 * kIters * kChains;  // wave-instructions of the op
  const double simds = 4.0 * ncu;
  const double cyc = best * 1e-3 * clock_khz * 1e3 * simds / winst;
  printf("{\"op\": \"%s\", \"ms\": %.4f, \"cycles_per_wave_instr_per_simd_at_peak_clock\": %.2f}\n",
         kName[OP], best, cyc);
  fflush(stdout);
}

int main() {
  hipDeviceProp_t p;
  CK(hipGetDeviceProperties(&p, 0));
  unsigned *in, *out;
  CK(hipMalloc(&in, 128 * 4));
  CK(hipMalloc(&out, 256 * 4));
  unsigned h[128];
  for (int i = 0; i < 128; ++i) h[i] = 0x01020304u * (i + 1);
  CK(hipMemcpy(in, h, sizeof h, hipMemcpyHostToDevice));
  printf("{\"cus\": %d, \"clock_khz\": %d}\n", p.multiProcessorCount, p.clockRate);
  run<0>(in, out, p.multiProcessorCount, p.clockRate);
  run<1>(in, out, p.multiProcessorCount, p.clockRate);
  run<2>(in, out, p.multiProcessorCount, p.clockRate);
  run<3>(in, out, p.multiProcessorCount, p.clockRate);
  run<4>(in, out, p.multiProcessorCount, p.clockRate);
  run<5>(in, out, p.multiProcessorCount, p.clockRate);
  run<6>(in, out, p.multiProcessorCount, p.clockRate);
  run<7>(in, out, p.multiProcessorCount, p.clockRate);
  run<8>(in, out, p.multiProcessorCount, p.clockRate);
  run<9>(in, out, p.multiProcessorCount, p.clockRate);
  run<10>(in, out, p.multiProcessorCount, p.clockRate);
  run<11>(in, out, p.multiProcessorCount, p.clockRate);
  run<12>(in, out, p.multiProcessorCount, p.clockRate);
  run<13>(in, out, p.multiProcessorCount, p.clockRate);
  run<14>(in, out, p.multiProcessorCount, p.clockRate);
  run<15>(in, out, p.multiProcessorCount, p.clockRate);
  run<16>(in, out, p.multiProcessorCount, p.clockRate);
  run<17>(in, out, p.multiProcessorCount, p.clockRate);
  run<18>(in, out, p.multiProcessorCount, p.clockRate);
  run<19>(in, out, p.multiProcessorCount, p.clockRate);
  run<20>(in, out, p.multiProcessorCount, p.clockRate);
  run<21>(in, out, p.multiProcessorCount, p.clockRate);
  run<22>(in, out, p.multiProcessorCount, p.clockRate);
  return 0;
}
