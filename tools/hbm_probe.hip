// hbm_probe.hip — MEASUREMENT TOOL, not part of the product library: the
// pure-read rate of a device buffer on this box (bench.py's per-box
// reference beside a reduce's bandwidth, roofline.box_read_probe).  Built by
// __graft_entry__.build() into build/libbldp_probe.so; loaded only by
// bench.py and tools/hbm_probe.py.
//
// k_read_probe: chunks of NL*256 16-byte words, each thread NL 16-byte loads
// (non-temporal unless PLAIN) at a 256-word stride, nothing stored (a store
// that never happens keeps the loads); one workgroup per chunk or wg_per_cu
// persistent workgroups per CU.  SLABS: the buffer is cut into NL equal slabs
// and chunk c reads 256 words of each (NL streams far apart at once, as a
// reduce reads a block's time rows).
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

namespace {
constexpr int kBlock = 256;
typedef float f4v __attribute__((ext_vector_type(4)));
int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }

template <bool PLAIN, int NL, bool SLABS>
__global__ __launch_bounds__(kBlock) void k_read_probe(const float *in, int64_t nchunk, int64_t n4,
                                                        int64_t slab, float *sink) {
  const int t = threadIdx.x;
  f4v acc = {0, 0, 0, 0};
  const f4v *p = reinterpret_cast<const f4v *>(in);
  for (int64_t c = blockIdx.x; c < nchunk; c += gridDim.x) {
    const int64_t b = SLABS ? c * kBlock + t : c * NL * kBlock + t;
    f4v v[NL];
#pragma unroll
    for (int k = 0; k < NL; ++k) {
      const int64_t i = b + (SLABS ? slab : kBlock) * k;
      v[k] = i >= n4 ? f4v{0, 0, 0, 0} : PLAIN ? p[i] : __builtin_nontemporal_load(p + i);
    }
#pragma unroll
    for (int k = 0; k < NL; ++k) acc += v[k];
  }
  if (acc.x == 1234.5f && sink) sink[t] = acc.y;
}

template <bool PLAIN, int NL, bool SLABS>
void go(const float *in, int64_t bytes, int wg_per_cu, int num_cus, hipStream_t s, hipEvent_t ev0,
        hipEvent_t ev1) {
  const int64_t n4 = bytes / 16, slab = cdiv(cdiv(n4, NL), kBlock) * kBlock;
  const int64_t nchunk = SLABS ? slab / kBlock : cdiv(n4, (int64_t)NL * kBlock);
  if (nchunk == 0) return;
  const int64_t grid = wg_per_cu > 0 ? std::min<int64_t>(nchunk, (int64_t)wg_per_cu * num_cus)
                                     : std::min<int64_t>(nchunk, INT32_MAX);
  if (ev1)  // events carried by the dispatch itself (as bldp_reduce_launch_timed)
    hipExtLaunchKernelGGL((k_read_probe<PLAIN, NL, SLABS>), dim3((unsigned)grid), dim3(kBlock), 0,
                          s, ev0, ev1, 0, in, nchunk, n4, slab, (float *)nullptr);
  else
    hipLaunchKernelGGL((k_read_probe<PLAIN, NL, SLABS>), dim3((unsigned)grid), dim3(kBlock), 0, s,
                       in, nchunk, n4, slab, (float *)nullptr);
}

template <bool SLABS>
void form_go(const float *in, int64_t bytes, int form, int num_cus, hipStream_t s, hipEvent_t ev0,
             hipEvent_t ev1) {
  const int g = form & 255;
  switch (form >> 8 & 3) {
    case 0: go<false, 16, SLABS>(in, bytes, g, num_cus, s, ev0, ev1); break;
    case 1: go<true, 16, SLABS>(in, bytes, g, num_cus, s, ev0, ev1); break;
    case 2: go<false, 8, SLABS>(in, bytes, g, num_cus, s, ev0, ev1); break;
    default: go<true, 8, SLABS>(in, bytes, g, num_cus, s, ev0, ev1); break;
  }
}
}  // namespace

// form: bits 0-7 workgroups per CU (0: one workgroup per chunk), bit 8 plain
// loads instead of non-temporal ones, bit 9 8 loads in flight per thread
// instead of 16, bit 10 slab-spread chunks.  ev_start/ev_stop: hipEvent_t or
// NULL.  Returns 0, or -1 for a bad argument / failed launch.
extern "C" __attribute__((visibility("default"))) int bldp_probe_read(const void *dev, int64_t bytes,
                                                                      int form, void *stream,
                                                                      void *ev_start,
                                                                      void *ev_stop) {
  if (bytes < 0 || form < 0 || form >= 2048) return -1;
  if (bytes >= 16 && (!dev || (uintptr_t)dev % 16)) return -1;
  int d = 0, ncu = 256;
  if (hipGetDevice(&d) != hipSuccess ||
      hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, d) != hipSuccess)
    ncu = 256;
  const float *in = static_cast<const float *>(dev);
  if (form & 1024)
    form_go<true>(in, bytes, form, ncu, (hipStream_t)stream, (hipEvent_t)ev_start,
                  (hipEvent_t)ev_stop);
  else
    form_go<false>(in, bytes, form, ncu, (hipStream_t)stream, (hipEvent_t)ev_start,
                   (hipEvent_t)ev_stop);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
