// mix_ceiling.hip — what a streaming kernel can reach on MI355X when it reads
// R bytes for every byte it writes (the read:write mix of fqav at fqavby = R
// with no time integration: F floats in, 1 out), at the sizes the reduce
// actually runs at (one 0002 file, the 0002 band, the 0000 band).
//
// k_mix<R>: a workgroup chunk is UB units; a unit is R x 4 KiB read
// contiguously (thread t reads float4 t + 256 k, k < R: every
// workgroup-instruction reads 4 KiB contiguous) and one 4 KiB contiguous write
// (thread t writes the sum of its R float4).  ~16 loads in flight per lane.
// This is the best case for the mix: every read and every write instruction
// covers whole 128-byte lines, writes are 1 KiB per wave-instruction.
//
//   hipcc --offload-arch=gfx950 -O3 -o build/mix_ceiling tools/mix_ceiling.hip
//   ./build/mix_ceiling [reps]          (JSON lines on stdout)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

typedef float f4v __attribute__((ext_vector_type(4)));

#define CK(x)                                                                    \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) {                                                      \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                   \
    }                                                                            \
  } while (0)

// ST: 1 = nt store, 2 = plain store, 0 = no store (pure read; the store is
// kept behind an impossible condition so the loads are not dead)
// LIF: float4 loads in flight per lane (16; 8 = the kurtosis kernels' batch)
template <int R, int ST, int LIF = 16>
__global__ __launch_bounds__(256) void k_mix(const f4v *__restrict__ in, f4v *__restrict__ out,
                                             int64_t nunits) {
  constexpr int UB = R >= LIF ? 1 : LIF / R;  // units per chunk
  constexpr int KB = R >= LIF ? LIF : R;      // loads per batch per unit
  const int t = threadIdx.x;
  const int64_t nchunks = (nunits + UB - 1) / UB;
  for (int64_t c = blockIdx.x; c < nchunks; c += gridDim.x) {
    const int64_t u0 = c * UB;
    f4v acc[UB];
#pragma unroll
    for (int b = 0; b < UB; ++b) acc[b] = f4v{0, 0, 0, 0};
#pragma unroll
    for (int k0 = 0; k0 < R; k0 += KB) {
      f4v v[UB * KB];
#pragma unroll
      for (int b = 0; b < UB; ++b)
#pragma unroll
        for (int k = 0; k < KB; ++k)
          v[b * KB + k] = (u0 + b < nunits)
                              ? __builtin_nontemporal_load(in + (u0 + b) * R * 256 + 256 * (k0 + k) + t)
                              : f4v{0, 0, 0, 0};
#pragma unroll
      for (int b = 0; b < UB; ++b)
#pragma unroll
        for (int k = 0; k < KB; ++k) acc[b] += v[b * KB + k];
    }
#pragma unroll
    for (int b = 0; b < UB; ++b) {
      if (u0 + b >= nunits) break;
      f4v *o = out + (u0 + b) * 256 + t;
      if (ST == 1) {
        __builtin_nontemporal_store(acc[b], o);
      } else if (ST == 2) {
        *o = acc[b];
      } else if (ST == 3) {  // the same 4 KiB as 4 dword stores per lane, 256 B per wave-instruction
        float *of = reinterpret_cast<float *>(out + (u0 + b) * 256);
        __builtin_nontemporal_store(acc[b].x, of + t);
        __builtin_nontemporal_store(acc[b].y, of + 256 + t);
        __builtin_nontemporal_store(acc[b].z, of + 512 + t);
        __builtin_nontemporal_store(acc[b].w, of + 768 + t);
      } else if (acc[b].x == 1234.5f) {
        *o = acc[b];
      }
    }
  }
}

struct Size {
  const char *label;
  int64_t bytes;
};

static float median(std::vector<float> v) {
  std::sort(v.begin(), v.end());
  return v[v.size() / 2];
}

// k_coltile<W, NW, NR>: the read pattern of the kurtosis register kernels
// (k_kurt_mid2: W = 8 bytes per lane, NW = 8 waves): a workgroup owns a
// (64 x W bytes) x nt column tile of one (nc x nt) bank, its NW waves split
// the nt rows, every wave-instruction reads 64 x W contiguous bytes at the
// row pitch; no arithmetic beyond a sum, one double per channel written (the
// kurtosis output).  Floor of that access pattern, not of the kernel.
template <int W, int NW, int NR>
__global__ __launch_bounds__(64 * NW) void k_coltile(const float *__restrict__ in,
                                                     double *__restrict__ out, int nc, int nt) {
  typedef float vt __attribute__((ext_vector_type(W / 4)));
  constexpr int CPW = 16 * W;  // channels per tile
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int ctiles = nc / CPW;
  const int ib = blockIdx.x / ctiles, c = (blockIdx.x % ctiles) * CPW + lane * (W / 4);
  const int r0 = __builtin_amdgcn_readfirstlane((wave * nt) / NW);
  const int cnt = __builtin_amdgcn_readfirstlane((((wave + 1) * nt) / NW) - r0);
  const float *p = in + (int64_t)ib * nc * nt + (int64_t)r0 * nc + c;
  vt v[NR];
#pragma unroll
  for (int r = 0; r < NR; ++r)
    v[r] = r < cnt ? __builtin_nontemporal_load(reinterpret_cast<const vt *>(p + (int64_t)r * nc)) : vt{};
  vt s = {};
#pragma unroll
  for (int r = 0; r < NR; ++r) s += v[r];
  __shared__ vt part[NW][64];
  part[wave][lane] = s;
  __syncthreads();
  if (wave == 0) {
    vt t = {};
#pragma unroll
    for (int q = 0; q < NW; ++q) t += part[q][lane];
    double *o = out + (int64_t)ib * nc + c;
#pragma unroll
    for (int k = 0; k < W / 4; ++k) o[k] = (double)t[k];
  }
}

template <int W, int NW, int NR>
static void run_coltile(const float *in, double *out, int nrow, int nc, int nt, int reps) {
  const unsigned grid = (unsigned)(nrow * (nc / (16 * W)));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::vector<float> ms;
  for (int r = 0; r < reps + 2; ++r) {
    CK(hipEventRecord(e0, 0));
    for (int i = 0; i < 5; ++i)
      hipLaunchKernelGGL((k_coltile<W, NW, NR>), dim3(grid), dim3(64 * NW), 0, 0, in, out, nc, nt);
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float m;
    CK(hipEventElapsedTime(&m, e0, e1));
    if (r >= 2) ms.push_back(m / 5);
  }
  const double rb = (double)nrow * nc * nt * 4, wb = (double)nrow * nc * 8;
  const float med = median(ms);
  printf("{\"size\": \"coltile %d x %d x %d\", \"bytes_per_lane\": %d, \"waves\": %d, \"rows_per_wave\": %d, "
         "\"read_bytes\": %.0f, \"write_bytes\": %.0f, \"ms_median\": %.4f, \"ms_min\": %.4f, "
         "\"GBps_median\": %.1f}\n",
         nrow, nc, nt, W, NW, NR, rb, wb, med, *std::min_element(ms.begin(), ms.end()),
         (rb + wb) / med / 1e6);
  fflush(stdout);
  CK(hipEventDestroy(e0));
  CK(hipEventDestroy(e1));
}

__global__ void k_fill(f4v *p, int64_t n4) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256)
    p[i] = f4v{1.f, 2.f, 3.f, 4.f};
}

template <int R, int ST, int LIF = 16>
static void run(const f4v *in, f4v *out, int64_t read_bytes, int grid_mode, int reps,
                const char *label, int ncu) {
  const int64_t nunits = read_bytes / ((int64_t)R * 4096);
  if (nunits <= 0) return;
  constexpr int UB = R >= LIF ? 1 : LIF / R;
  const int64_t nchunks = (nunits + UB - 1) / UB;
  // grid_mode 0: one workgroup per chunk; k > 0: k workgroups per CU (persistent)
  const int64_t grid = grid_mode == 0 ? nchunks : std::min<int64_t>(nchunks, (int64_t)grid_mode * ncu);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::vector<float> ms;
  for (int r = 0; r < reps + 2; ++r) {
    CK(hipEventRecord(e0, 0));
    for (int i = 0; i < 5; ++i)  // back to back, as the library's timings are taken
      hipLaunchKernelGGL((k_mix<R, ST, LIF>), dim3((unsigned)grid), dim3(256), 0, 0, in, out, nunits);
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float m;
    CK(hipEventElapsedTime(&m, e0, e1));
    if (r >= 2) ms.push_back(m / 5);
  }
  const double rb = (double)nunits * R * 4096, wb = ST ? (double)nunits * 4096 : 0.0;
  const float med = median(ms);
  printf("{\"size\": \"%s\", \"read_bytes\": %.0f, \"write_bytes\": %.0f, \"R\": %d, "
         "\"loads_in_flight\": %d, \"store\": \"%s\", "
         "\"grid\": \"%s\", \"ms_median\": %.4f, \"ms_min\": %.4f, \"GBps_median\": %.1f}\n",
         label, rb, wb, R, LIF, ST == 1 ? "nt" : ST == 2 ? "plain" : ST == 3 ? "nt dword" : "none",
         grid_mode == 0 ? "chunk" : (grid_mode == 1 ? "1/CU" : grid_mode == 2 ? "2/CU" : "4/CU"),
         med, *std::min_element(ms.begin(), ms.end()), (rb + wb) / med / 1e6);
  fflush(stdout);
  CK(hipEventDestroy(e0));
  CK(hipEventDestroy(e1));
}

template <int R>
static void run_r(const f4v *in, f4v *out, int64_t bytes, int reps, const char *label, int ncu,
                  bool grids) {
  run<R, 1>(in, out, bytes, 0, reps, label, ncu);
  run<R, 2>(in, out, bytes, 0, reps, label, ncu);
  if (grids)
    for (int g : {1, 2, 4}) run<R, 1>(in, out, bytes, g, reps, label, ncu);
}

int main(int argc, char **argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 20;
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  const int ncu = prop.multiProcessorCount;
  const int64_t big = 32ll << 30;
  f4v *in, *out;
  CK(hipMalloc(&in, big));
  CK(hipMalloc(&out, big));  // R = 1 (copy) writes as much as it reads
  hipLaunchKernelGGL(k_fill, dim3(65536), dim3(256), 0, 0, in, big / 16);
  CK(hipDeviceSynchronize());
  if (argc > 2 && std::string(argv[2]) == "dword") {  // store width at the 0002 band size
    const int64_t b2 = 8ll * 65536 * 279 * 4;
    for (int ST : {1, 3}) {
      const char *l = "0002 band 585 MB";
      if (ST == 1) {
        run<2, 1>(in, out, b2, 0, reps, l, ncu); run<3, 1>(in, out, b2, 0, reps, l, ncu);
        run<4, 1>(in, out, b2, 0, reps, l, ncu); run<12, 1>(in, out, b2, 0, reps, l, ncu);
      } else {
        run<2, 3>(in, out, b2, 0, reps, l, ncu); run<3, 3>(in, out, b2, 0, reps, l, ncu);
        run<4, 3>(in, out, b2, 0, reps, l, ncu); run<12, 3>(in, out, b2, 0, reps, l, ncu);
      }
    }
    return 0;
  }
  if (argc > 2 && std::string(argv[2]) == "kurt") {
    // the Float32 kurtosis bands' mixes: cfg3 reads 32 GiB
    // and writes 4 GiB of Float64 (R = 8), cfg4 reads 14.4 GB (pure read), cfg2
    // 585 MB (pure read); every grid form, 16 and 8 float4 loads in flight
    const Size ks[] = {{"0000 band 32 GiB", big}, {"0001 band 14.4 GB", 8ll * 512 * 879616 * 4},
                       {"0002 band 585 MB", 8ll * 65536 * 279 * 4}};
    for (const Size &s : ks) {
      if (s.bytes == big) {
        for (int g : {0, 1, 2, 4}) {
          run<8, 1, 16>(in, out, s.bytes, g, reps, s.label, ncu);
          run<8, 1, 8>(in, out, s.bytes, g, reps, s.label, ncu);
        }
        run<8, 2, 16>(in, out, s.bytes, 0, reps, s.label, ncu);
      }
      for (int g : {0, 1, 2, 4}) {
        run<16, 0, 16>(in, out, s.bytes, g, reps, s.label, ncu);
        run<8, 0, 8>(in, out, s.bytes, g, reps, s.label, ncu);
      }
    }
    return 0;
  }
  if (argc > 2 && std::string(argv[2]) == "coltile") {  // the 0002 band as the kurtosis reads it
    const float *fi = reinterpret_cast<const float *>(in);
    double *fo = reinterpret_cast<double *>(out);
    for (int nt : {279, 272}) {
      run_coltile<8, 8, 35>(fi, fo, 8, 65536, nt, reps);    // k_kurt_mid2's geometry
      run_coltile<8, 4, 70>(fi, fo, 8, 65536, nt, reps);
      run_coltile<16, 8, 35>(fi, fo, 8, 65536, nt, reps);
      run_coltile<16, 16, 18>(fi, fo, 8, 65536, nt, reps);
      run_coltile<8, 16, 18>(fi, fo, 8, 65536, nt, reps);
      run_coltile<4, 8, 35>(fi, fo, 8, 65536, nt, reps);    // k_kurt_mid's 256 B per wave
    }
    return 0;
  }
  // one 0002 file (65536 x 279 floats), the 0002 band (8 of them), the 0000 band
  const Size all_sizes[] = {{"0002 file 73 MB", 65536ll * 279 * 4},
                            {"0002 band 585 MB", 8ll * 65536 * 279 * 4},
                            {"0001 band 14.4 GB", 8ll * 512 * 879616 * 4},
                            {"0000 band 32 GiB", big}};
  // argv[2] = "0001" / "0002": only that product's sizes
  const std::string only = argc > 2 ? std::string(argv[2]) : std::string();
  std::vector<Size> sizes;
  for (const Size &z : all_sizes)
    if (only.empty() || std::string(z.label).rfind(only, 0) == 0) sizes.push_back(z);
  for (const Size &s : sizes) {
    const bool grids = s.bytes < (1ll << 30);
    run_r<1>(in, out, s.bytes, reps, s.label, ncu, grids);
    run_r<2>(in, out, s.bytes, reps, s.label, ncu, grids);
    run_r<3>(in, out, s.bytes, reps, s.label, ncu, grids);
    run_r<4>(in, out, s.bytes, reps, s.label, ncu, grids);
    run_r<8>(in, out, s.bytes, reps, s.label, ncu, grids);
    run_r<12>(in, out, s.bytes, reps, s.label, ncu, grids);
    run_r<16>(in, out, s.bytes, reps, s.label, ncu, grids);
    run_r<64>(in, out, s.bytes, reps, s.label, ncu, grids);
    run_r<256>(in, out, s.bytes, reps, s.label, ncu, grids);
    run<16, 0>(in, out, s.bytes, 0, reps, s.label, ncu);  // pure read, 64 KiB per workgroup
    if (grids)
      for (int g : {1, 2, 4}) run<16, 0>(in, out, s.bytes, g, reps, s.label, ncu);
  }
  CK(hipFree(in));
  CK(hipFree(out));
  return 0;
}
