// hbm_ceiling.hip — what read bandwidth can a gfx950 streaming kernel reach?
//
// Measurement tool (not product code).  Sweeps pure-read kernels over a
// 32 GiB buffer (the cfg3 band size, far beyond the 256 MiB Infinity Cache):
// access shape (contiguous per workgroup / per wave / the cfg3 row pattern),
// loads in flight per lane, workgroup chunk size, persistent vs one-shot grid,
// and the load cache policy (plain, nt, buffer loads with sc0/sc1/nt bits).
// Every kernel folds what it reads into one float per workgroup, so nothing
// is optimised away and writes are negligible.  Prints one JSON line per
// variant: best and median GB/s over the timed launches.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/hbm_ceiling.hip -o build/hbm_ceiling
//   build/hbm_ceiling [GiB [reps [path/to/libbldp_hip.so]]]
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <dlfcn.h>

#include <algorithm>
#include <string>
#include <vector>

#define CK(x)                                                                      \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));     \
      exit(1);                                                                     \
    }                                                                              \
  } while (0)

typedef float f4v __attribute__((ext_vector_type(4)));

// load policies
enum { P_PLAIN = 0, P_NT = 1, P_BUF = 2, P_BUF_NT = 3, P_BUF_SC1 = 4, P_BUF_SC0SC1 = 5,
       P_BUF_NTSC1 = 6 };

template <int POL>
__device__ __forceinline__ f4v ld(const f4v *base, __amdgpu_buffer_rsrc_t rs, int64_t idx) {
  if constexpr (POL == P_PLAIN) return base[idx];
  else if constexpr (POL == P_NT) return __builtin_nontemporal_load(base + idx);
  else {
    constexpr int aux = POL == P_BUF ? 0 : POL == P_BUF_NT ? 2 : POL == P_BUF_SC1 ? 16
                      : POL == P_BUF_SC0SC1 ? 17 : 18;
    return __builtin_bit_cast(f4v, __builtin_amdgcn_raw_buffer_load_b128(
                                        rs, (int)(idx * 16), 0, aux));
  }
}

__device__ __forceinline__ float fold(f4v v) { return (v.x + v.y) + (v.z + v.w); }

// (1) each workgroup reads `chunk4` float4 contiguous, a workgroup-instruction
// covers 4 KiB, B loads in flight per lane.  Persistent when gridDim < nchunks.
template <int B, int POL>
__global__ __launch_bounds__(256) void k_contig(const f4v *in, int64_t nchunks, int64_t chunk4,
                                                float *out) {
  float s = 0.f;
  for (int64_t c = blockIdx.x; c < nchunks; c += gridDim.x) {
    const f4v *base = in + c * chunk4;
    __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc((void *)base, 0, (int)(chunk4 * 16), 0x00020000);
    f4v acc[B];
#pragma unroll
    for (int u = 0; u < B; ++u) acc[u] = f4v{0, 0, 0, 0};
    for (int64_t k = threadIdx.x; k < chunk4; k += 256 * B) {
      f4v v[B];
#pragma unroll
      for (int u = 0; u < B; ++u) v[u] = ld<POL>(base, rs, k + u * 256);
#pragma unroll
      for (int u = 0; u < B; ++u) acc[u] += v[u];
    }
#pragma unroll
    for (int u = 1; u < B; ++u) acc[0] += acc[u];
    s += fold(acc[0]);
  }
  if (s == 1234.5f) out[blockIdx.x] = s;  // never true on this data; keeps the loads live
}

// (2) each wave reads its own contiguous span (1 KiB per wave-instruction).
template <int B, int POL>
__global__ __launch_bounds__(256) void k_wave(const f4v *in, int64_t chunk4, float *out) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t span4 = chunk4 / 4;
  const f4v *base = in + blockIdx.x * chunk4 + wave * span4;
  __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc((void *)base, 0, (int)(span4 * 16), 0x00020000);
  f4v acc[B];
#pragma unroll
  for (int u = 0; u < B; ++u) acc[u] = f4v{0, 0, 0, 0};
  for (int64_t k = lane; k < span4; k += 64 * B) {
    f4v v[B];
#pragma unroll
    for (int u = 0; u < B; ++u) v[u] = ld<POL>(base, rs, k + u * 64);
#pragma unroll
    for (int u = 0; u < B; ++u) acc[u] += v[u];
  }
#pragma unroll
  for (int u = 1; u < B; ++u) acc[0] += acc[u];
  float s = fold(acc[0]);
  if (s == 1234.5f) out[blockIdx.x] = s;
}

// (3) the cfg3 shape: nrow rows of row4 float4 (rows 256 MiB apart for one
// bank); a workgroup owns a 16 KiB column segment of every row of its bank.
// IL=false: each wave streams its own 4 KiB of the segment (one 1024-channel
// group, what k_reduce_vec does); IL=true: wave-instructions interleave so a
// workgroup-instruction covers 4 KiB contiguous.  RB rows x 4 float4 in
// flight per lane.  Persistent when gridDim < tiles.
template <int POL, bool IL, int RB, int EPI = 0>
__global__ __launch_bounds__(256) void k_cfg3(const f4v *in, int64_t row4, int nrow,
                                              int64_t segs_per_bank, int64_t ntiles, float *out) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float s = 0.f;
  for (int64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const int64_t bank = t / segs_per_bank, seg = t % segs_per_bank;
    const f4v *base = in + bank * row4 * nrow + seg * 1024 + (IL ? wave * 64 : wave * 256) + lane;
    f4v acc[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) acc[u] = f4v{0, 0, 0, 0};
    for (int r = 0; r < nrow; r += RB) {
      f4v v[RB * 4];
#pragma unroll
      for (int u = 0; u < RB; ++u)
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const f4v *p = base + (int64_t)(r + u) * row4 + k * (IL ? 256 : 64);
          v[u * 4 + k] = POL == P_NT ? __builtin_nontemporal_load(p) : *p;
        }
#pragma unroll
      for (int u = 0; u < RB * 4; ++u) acc[u % 8] += v[u];
    }
#pragma unroll
    for (int u = 1; u < 8; ++u) acc[0] += acc[u];
    if constexpr (EPI == 1) {  // k_reduce_il's epilogue: lane fold, LDS, barrier, store
      __shared__ float red[4][4];
      float x = fold(acc[0]);
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) x += __shfl_xor(x, off, 64);
      if (lane == 0) red[wave][0] = x;
      __syncthreads();
      if (threadIdx.x < 4) out[t * 4 + threadIdx.x] = red[0][0] + red[threadIdx.x][0];
    } else {
      s += fold(acc[0]);
    }
  }
  if (EPI == 0 && s == 1234.5f) out[blockIdx.x] = s;
}

// (3b) the cfg3 shape, software-pipelined over the tiles of a persistent
// workgroup: the epilogue of tile k (lane fold, cross-wave LDS combine when
// interleaved, store) runs while the first loads of tile k+1 are in flight.
// IL as above; the barrier carries no fence, so it waits on LDS only.
__device__ __forceinline__ void lds_barrier() {
  __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0); vmcnt/expcnt untouched
  __builtin_amdgcn_s_barrier();
}
template <bool IL>
__device__ __forceinline__ void epi(f4v a0, int lane, int wave, float (*red)[4], float *out,
                                    int64_t t) {
  float x = fold(a0);
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) x += __shfl_xor(x, off, 64);
  if (IL) {
    if (lane == 0) red[wave][0] = x;
    lds_barrier();
    if (threadIdx.x < 4) out[t * 4 + threadIdx.x] = red[0][0] + red[threadIdx.x][0];
  } else if (lane == 0) {
    out[t * 4 + wave] = x;
  }
}
template <bool IL>
__global__ __launch_bounds__(256) void k_cfg3_pipe(const f4v *in, int64_t row4, int nrow,
                                                   int64_t segs_per_bank, int64_t ntiles,
                                                   float *out) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  __shared__ float red[2][4][4];
  f4v prev = f4v{0, 0, 0, 0};
  int64_t prev_t = -1;
  int par = 0;
  for (int64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const int64_t bank = t / segs_per_bank, seg = t % segs_per_bank;
    const f4v *base = in + bank * row4 * nrow + seg * 1024 + (IL ? wave * 64 : wave * 256) + lane;
    f4v acc[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) acc[u] = f4v{0, 0, 0, 0};
    for (int r = 0; r < nrow; r += 2) {
      f4v v[8];
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int k = 0; k < 4; ++k)
          v[u * 4 + k] = __builtin_nontemporal_load(base + (int64_t)(r + u) * row4 +
                                                    k * (IL ? 256 : 64));
      if (r == 0 && prev_t >= 0) {
        epi<IL>(prev, lane, wave, red[par], out, prev_t);
        par ^= 1;
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) acc[u] += v[u];
    }
#pragma unroll
    for (int u = 1; u < 8; ++u) acc[0] += acc[u];
    prev = acc[0];
    prev_t = t;
  }
  if (prev_t >= 0) epi<IL>(prev, lane, wave, red[par], out, prev_t);
}

// (3c) the kurtosis shape: one float4 column per lane over nrow rows (4 KiB
// per workgroup per row), then 32 B of output per lane written as two 1 KiB
// contiguous wave-instructions (STORE 1 = nt, 2 = plain, 0 = none): 1 byte
// written per 8 read, what k_kurt_regs does on the 0000 product.
template <int STORE>
__global__ __launch_bounds__(256) void k_kmix(const f4v *in, int64_t row4, int nrow,
                                              int64_t segs_per_bank, f4v *out) {
  const int lane = threadIdx.x & 63;
  const int64_t bank = blockIdx.x / segs_per_bank, seg = blockIdx.x % segs_per_bank;
  const f4v *base = in + bank * row4 * nrow + seg * 256 + threadIdx.x;
  f4v v[16];
#pragma unroll
  for (int r = 0; r < 16; ++r)
    v[r] = r < nrow ? __builtin_nontemporal_load(base + (int64_t)r * row4) : f4v{0, 0, 0, 0};
  f4v a = v[0];
#pragma unroll
  for (int r = 1; r < 16; ++r) a += v[r] * v[r];
  f4v *o = out + (int64_t)blockIdx.x * 512 + (threadIdx.x >> 6) * 128;
  if (STORE >= 10) {  // buffer stores with cache-policy bits STORE - 10
    __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void *)o, 0, 128 * 16,
                                                                  0x00020000);
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned, a),
                                           rs, lane * 16, 0, STORE - 10);
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned, a * 2.f),
                                           rs, (64 + lane) * 16, 0, STORE - 10);
  } else if (STORE == 1) {
    __builtin_nontemporal_store(a, o + lane);
    __builtin_nontemporal_store(a * 2.f, o + 64 + lane);
  } else if (STORE == 2) {
    o[lane] = a;
    o[64 + lane] = a * 2.f;
  } else if (a.x == 1234.5f) {
    o[lane] = a;
  }
}

// (3e) the time-integration shape (fqavby = 1, tavby = 16, k_reduce_narrow):
// one float4 column per lane over nrow rows, then ONE float4 of output per
// lane (1 byte written per 16 read) as a 1 KiB wave-instruction; 8 rows in
// flight.  STORE 1 = nt, 2 = plain.
template <int STORE>
__global__ __launch_bounds__(256) void k_nmix(const f4v *in, int64_t row4, int nrow,
                                              int64_t segs_per_bank, f4v *out) {
  const int64_t bank = blockIdx.x / segs_per_bank, seg = blockIdx.x % segs_per_bank;
  const f4v *base = in + bank * row4 * nrow + seg * 256 + threadIdx.x;
  f4v a = f4v{0, 0, 0, 0}, b = a;
  for (int r = 0; r < nrow; r += 8) {
    f4v v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = __builtin_nontemporal_load(base + (int64_t)(r + u) * row4);
#pragma unroll
    for (int u = 0; u < 8; u += 2) {
      a += v[u];
      b += v[u + 1];
    }
  }
  f4v *o = out + (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (STORE == 1)
    __builtin_nontemporal_store(a + b, o);
  else
    *o = a + b;
}

// (3d) tail study: the interleaved cfg3 pattern with G 1024-channel groups
// per workgroup (4 KiB x G per row, 16 rows), on nbank banks.
template <int G>
__global__ __launch_bounds__(256) void k_cfg3g(const f4v *in, int64_t row4, int nrow,
                                               int64_t segs_per_bank, float *out) {
  const int64_t t = blockIdx.x;
  const int64_t bank = t / segs_per_bank, seg = t % segs_per_bank;
  const f4v *base = in + bank * row4 * nrow + seg * 256 * G + threadIdx.x;
  f4v acc[G];
#pragma unroll
  for (int g = 0; g < G; ++g) acc[g] = f4v{0, 0, 0, 0};
  constexpr int RB = G >= 8 ? 1 : 8 / G;
  for (int r = 0; r < nrow; r += RB) {
    f4v v[RB * G];
#pragma unroll
    for (int u = 0; u < RB; ++u)
#pragma unroll
      for (int g = 0; g < G; ++g)
        v[u * G + g] = __builtin_nontemporal_load(base + (int64_t)(r + u) * row4 + g * 256);
#pragma unroll
    for (int u = 0; u < RB * G; ++u) acc[u % G] += v[u];
  }
  float x = 0.f;
#pragma unroll
  for (int g = 0; g < G; ++g) x += fold(acc[g]);
  if (x == 1234.5f) out[t] = x;
}

__global__ void k_fill(f4v *p, int64_t n4) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256)
    p[i] = f4v{1.f, 2.f, 3.f, (float)(i & 7)};
}

struct Res {
  double best, med;
};

template <typename L>
Res timeit(L launch, double bytes, int reps) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  launch();
  launch();
  CK(hipDeviceSynchronize());
  std::vector<double> g;
  for (int r = 0; r < reps; ++r) {
    CK(hipEventRecord(a, 0));
    launch();
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    g.push_back(bytes / (ms * 1e-3) / 1e9);
  }
  CK(hipGetLastError());
  std::sort(g.begin(), g.end());
  CK(hipEventDestroy(a));
  CK(hipEventDestroy(b));
  return {g.back(), g[g.size() / 2]};
}

static void report(const char *name, Res r) {
  printf("{\"variant\": \"%s\", \"best_GBps\": %.1f, \"median_GBps\": %.1f}\n", name, r.best,
         r.med);
  fflush(stdout);
}

int main(int argc, char **argv) {
  const int64_t gib = argc > 1 ? atoll(argv[1]) : 32;
  const int reps = argc > 2 ? atoi(argv[2]) : 10;
  const int64_t bytes = gib << 30, n4 = bytes / 16;
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  f4v *in;
  float *out;
  CK(hipMalloc(&in, bytes));
  CK(hipMalloc(&out, 1 << 28));
  hipLaunchKernelGGL(k_fill, dim3(cus * 8), dim3(256), 0, 0, in, n4);
  CK(hipDeviceSynchronize());
  char name[160];

  const bool kmix_only = argc > 4 && std::string(argv[4]) == "kmix";
  if (argc > 4 && std::string(argv[4]) == "nmix" && gib == 32) {
    // (3e) read 32 GiB in the cfg3 row pattern + write 2 GiB (F = 1, T = 16)
    const int nrow = 16;
    const int64_t row4 = (1ll << 26) / 4, segs = row4 / 256;
    f4v *wout;
    CK(hipMalloc(&wout, 2ll << 30));
    const double mb = (double)bytes + (2ll << 30);
    report("narrow-shape read 32 GiB + write 2 GiB (1/16), nt stores",
           timeit([&] { hipLaunchKernelGGL((k_nmix<1>), dim3((unsigned)(segs * 8)), dim3(256), 0, 0,
                                           in, row4, nrow, segs, wout); }, mb, reps));
    report("narrow-shape read 32 GiB + write 2 GiB (1/16), plain stores",
           timeit([&] { hipLaunchKernelGGL((k_nmix<2>), dim3((unsigned)(segs * 8)), dim3(256), 0, 0,
                                           in, row4, nrow, segs, wout); }, mb, reps));
    if (argc > 3) {  // the library's narrow path on the same buffer
      void *h = dlopen(argv[3], RTLD_NOW);
      typedef int (*band_fn)(int, const float *const *, int64_t, int64_t, int64_t, const int64_t *,
                             int64_t, int64_t, int, float *, void *);
      band_fn f = h ? (band_fn)dlsym(h, "bldp_band_reduce_f32") : nullptr;
      if (f) {
        const float *banks[8];
        for (int b = 0; b < 8; ++b) banks[b] = (const float *)in + (int64_t)b * (1ll << 30);
        report("libbldp band reduce, F=1 T=16 (k_reduce_narrow), same buffer",
               timeit([&] {
                 if (f(8, banks, 1ll << 26, 1, 16, nullptr, 1, 16, 0, (float *)wout, nullptr)) exit(2);
               }, mb, reps));
      }
    }
    CK(hipFree(wout));
    CK(hipFree(in));
    CK(hipFree(out));
    return 0;
  }
  if (kmix_only) goto kmix;
  // (1) contiguous per workgroup: chunk size x loads in flight x policy
#define CONTIG(B, POL, CHUNK_KIB, GRID_PER_CU)                                             \
  {                                                                                        \
    const int64_t chunk4 = (int64_t)(CHUNK_KIB) * 1024 / 16, nch = n4 / chunk4;            \
    const int64_t grid = (GRID_PER_CU) ? (int64_t)(GRID_PER_CU) * cus : nch;               \
    snprintf(name, sizeof name, "contig B=%d pol=%s chunk=%dKiB grid=%s%d", B, #POL,       \
             CHUNK_KIB, (GRID_PER_CU) ? "persistent x" : "one-shot ", GRID_PER_CU);        \
    report(name, timeit([&] { hipLaunchKernelGGL((k_contig<B, POL>), dim3((unsigned)grid), \
                                                 dim3(256), 0, 0, in, nch, chunk4, out); }, \
                        (double)nch * chunk4 * 16, reps));                                 \
  }
  CONTIG(8, P_PLAIN, 256, 0)
  CONTIG(8, P_NT, 256, 0)
  CONTIG(8, P_BUF, 256, 0)
  CONTIG(8, P_BUF_NT, 256, 0)
  CONTIG(8, P_BUF_SC1, 256, 0)
  CONTIG(8, P_BUF_SC0SC1, 256, 0)
  CONTIG(8, P_BUF_NTSC1, 256, 0)
  CONTIG(4, P_NT, 256, 0)
  CONTIG(16, P_NT, 256, 0)
  CONTIG(8, P_NT, 64, 0)
  CONTIG(8, P_NT, 1024, 0)
  CONTIG(8, P_NT, 4096, 0)
  CONTIG(8, P_NT, 256, 2)
  CONTIG(8, P_NT, 256, 4)
  CONTIG(8, P_NT, 256, 8)
  CONTIG(8, P_NT, 256, 16)
  CONTIG(16, P_BUF_NT, 1024, 0)

  // (2) contiguous per wave
#define WAVE(B, POL, CHUNK_KIB)                                                             \
  {                                                                                         \
    const int64_t chunk4 = (int64_t)(CHUNK_KIB) * 1024 / 16, nch = n4 / chunk4;             \
    snprintf(name, sizeof name, "wave-contig B=%d pol=%s wg_chunk=%dKiB", B, #POL, CHUNK_KIB); \
    report(name, timeit([&] { hipLaunchKernelGGL((k_wave<B, POL>), dim3((unsigned)nch),      \
                                                 dim3(256), 0, 0, in, chunk4, out); },       \
                        (double)nch * chunk4 * 16, reps));                                  \
  }
  WAVE(8, P_NT, 256)
  WAVE(8, P_PLAIN, 256)
  WAVE(16, P_NT, 256)

  // (3) the cfg3 row pattern: 8 banks x 16 rows x 2^26 floats (when 32 GiB)
  {
    const int nrow = 16;
    const int64_t nbank = gib / 4 > 0 ? gib / 4 : 1;
    const int64_t row4 = bytes / nbank / nrow / 16;
    const int64_t segs = row4 / 1024, ntiles = segs * nbank;
#define CFG3(POL, IL, RB, GRID_PER_CU, ...)                                                          \
    {                                                                                           \
      const int64_t grid = (GRID_PER_CU) ? (int64_t)(GRID_PER_CU) * cus : ntiles;               \
      snprintf(name, sizeof name, "cfg3-pattern pol=%s interleave=%d rows_in_flight=%d grid=%s%d %s", \
               #POL, (int)(IL), RB, (GRID_PER_CU) ? "persistent x" : "one-shot ", GRID_PER_CU, \
               #__VA_ARGS__);                                                                  \
      report(name, timeit([&] { hipLaunchKernelGGL((k_cfg3<POL, IL, RB __VA_OPT__(,) __VA_ARGS__>), dim3((unsigned)grid), \
                                                   dim3(256), 0, 0, in, row4, nrow, segs, ntiles, \
                                                   out); },                                     \
                          (double)bytes, reps));                                                \
    }
    CFG3(P_NT, false, 2, 0)
    CFG3(P_PLAIN, false, 2, 0)
    CFG3(P_NT, true, 2, 0)
    CFG3(P_NT, false, 1, 0)
    CFG3(P_NT, true, 1, 0)
    CFG3(P_NT, false, 4, 0)
    CFG3(P_NT, true, 4, 0)
    CFG3(P_NT, false, 2, 2)
    CFG3(P_NT, true, 2, 2)
    CFG3(P_NT, false, 2, 4)
    CFG3(P_NT, true, 2, 4)
    CFG3(P_NT, true, 1, 2)
    CFG3(P_NT, true, 4, 2)
    CFG3(P_NT, true, 2, 0, 1)
    CFG3(P_NT, false, 2, 0, 1)
#define PIPE(IL, GRID_PER_CU)                                                                  \
    {                                                                                          \
      const int64_t grid = (GRID_PER_CU) ? (int64_t)(GRID_PER_CU) * cus : ntiles;              \
      snprintf(name, sizeof name, "cfg3-pattern pipelined epilogue interleave=%d grid=%s%d",   \
               (int)(IL), (GRID_PER_CU) ? "persistent x" : "one-shot ", GRID_PER_CU);          \
      report(name, timeit([&] { hipLaunchKernelGGL((k_cfg3_pipe<IL>), dim3((unsigned)grid),    \
                                                   dim3(256), 0, 0, in, row4, nrow, segs,      \
                                                   ntiles, out); },                            \
                          (double)bytes, reps));                                               \
    }
    PIPE(true, 0)
    PIPE(false, 0)
    PIPE(true, 2)
    PIPE(true, 4)
    PIPE(true, 8)
    PIPE(false, 2)
    PIPE(false, 4)
    PIPE(false, 8)
  }
  // (3d) tail study: workgroup size x 1 / 8 banks of the cfg3 shape
  if (gib == 32 && argc > 4 && std::string(argv[4]) == "tail") {
    const int nrow = 16;
    const int64_t row4 = (1ll << 26) / 4;
    for (int nb : {1, 8}) {
#define TAILG(G)                                                                             \
      {                                                                                      \
        const int64_t segs = row4 / (256 * G);                                               \
        snprintf(name, sizeof name, "tail: %d bank(s), %d groups (%d KiB) per workgroup", nb, \
                 G, 64 * G);                                                                 \
        report(name, timeit([&] { hipLaunchKernelGGL((k_cfg3g<G>), dim3((unsigned)(segs * nb)), \
                                                     dim3(256), 0, 0, in, row4, nrow, segs, out); }, \
                            (double)nb * (4ll << 30), reps));                                \
      }
      TAILG(1) TAILG(2) TAILG(4) TAILG(8)
    }
    CK(hipFree(in));
    CK(hipFree(out));
    return 0;
  }

  // (3c) kurtosis-shaped read + 1/8 write mix
kmix:
  if (gib == 32) {
    const int nrow = 16;
    const int64_t row4 = (1ll << 26) / 4, segs = row4 / 256;
    f4v *wout;
    CK(hipMalloc(&wout, 4ll << 30));
    const double mb = (double)bytes + (4ll << 30);
    report("kurt-shape read 32 GiB + write 4 GiB, nt stores",
           timeit([&] { hipLaunchKernelGGL((k_kmix<1>), dim3((unsigned)(segs * 8)), dim3(256), 0, 0,
                                           in, row4, nrow, segs, wout); }, mb, reps));
    report("kurt-shape read 32 GiB + write 4 GiB, plain stores",
           timeit([&] { hipLaunchKernelGGL((k_kmix<2>), dim3((unsigned)(segs * 8)), dim3(256), 0, 0,
                                           in, row4, nrow, segs, wout); }, mb, reps));
#define KMIX(AUX, NAME)                                                                      \
    report("kurt-shape read 32 GiB + write 4 GiB, buffer stores " NAME,                      \
           timeit([&] { hipLaunchKernelGGL((k_kmix<10 + AUX>), dim3((unsigned)(segs * 8)),     \
                                           dim3(256), 0, 0, in, row4, nrow, segs, wout); }, mb, reps));
    KMIX(0, "plain") KMIX(2, "nt") KMIX(16, "sc1") KMIX(1, "sc0") KMIX(17, "sc0 sc1")
    KMIX(18, "nt sc1") KMIX(3, "nt sc0") KMIX(19, "nt sc0 sc1")
    report("kurt-shape read 32 GiB, no stores (bytes = read only)",
           timeit([&] { hipLaunchKernelGGL((k_kmix<0>), dim3((unsigned)(segs * 8)), dim3(256), 0, 0,
                                           in, row4, nrow, segs, wout); }, (double)bytes, reps));
    CK(hipFree(wout));
  }

  // (4) the library's own band launch on the same buffer (8 banks of 4 GiB
  // carved from it), when libbldp_hip.so is given as argv[3]
  if (argc > 3 && gib == 32) {
    void *h = dlopen(argv[3], RTLD_NOW);
    typedef int (*band_fn)(int, const float *const *, int64_t, int64_t, int64_t, const int64_t *,
                           int64_t, int64_t, int, float *, void *);
    band_fn f = h ? (band_fn)dlsym(h, "bldp_band_reduce_f32") : nullptr;
    if (!f) {
      fprintf(stderr, "no bldp_band_reduce_f32 in %s\n", argv[3]);
      return 1;
    }
    const float *banks[8];
    for (int b = 0; b < 8; ++b) banks[b] = (const float *)in + (int64_t)b * (1ll << 30);
    report("libbldp band reduce, F=1024 T=16, 8 x (2^26 x 1 x 16) in one allocation",
           timeit([&] {
             if (f(8, banks, 1ll << 26, 1, 16, nullptr, 1024, 16, 0, out, nullptr)) exit(2);
           }, (double)bytes + 8.0 * 65536 * 4, reps));
  }
  CK(hipFree(in));
  CK(hipFree(out));
  return 0;
}
