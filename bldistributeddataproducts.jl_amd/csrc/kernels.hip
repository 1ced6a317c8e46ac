// kernels.hip — CDNA4 (gfx950) kernels of libbldp_hip.
//
// The hot path is fqav (src/gbtworkerfunctions.jl:16-20) fused with the
// additive time integration (fqav on axis 3) over a window of a
// (nchan, nif, ntime) Float32 filterbank, channel fastest.  It is a pure HBM
// stream (<= 0.25 flop/byte), so the kernels are built around:
//   * 16-byte (global_load_dwordx4) loads along the channel axis, one 1 KiB
//     contiguous segment per wave-instruction;
//   * batches of 8 independent loads per lane before any use, with 8
//     independent accumulators (latency hiding + shorter FP32 add chains);
//   * wavefront xor-shuffles to combine the lanes of one decimation group;
//   * an LDS combine of the waves that split the time rows of one tile, and
//     a deterministic two-stage (partials + finalize) split of very long time
//     blocks across workgroups;
//   * IEEE-754-2019 maximum/minimum (v_maximum3_f32 / v_minimum3_f32 on
//     gfx950) for max/min, which is exactly Julia's max/min: NaN propagates
//     and -0.0 < +0.0.
// No MFMA: nothing here is matmul shaped.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include <atomic>
#include <cstring>

#include "bldp_impl.h"

namespace bldp {
namespace {

constexpr int kBlock = 256;  // 4 waves of 64
typedef float f4v __attribute__((ext_vector_type(4)));
// What the streaming loads point at: a float4 that may sit on any dword
// boundary (plan option unaligned_vec: windows off a 16-byte boundary).  gfx950
// executes global_load_dwordx4 at dword alignment, so the code is unchanged.
typedef float f4u __attribute__((ext_vector_type(4), aligned(4)));

template <int OP>
struct R {
  // sum and mean: Julia's reducedim init is zero(T) (+0.0f)
  __device__ static constexpr float id() { return 0.0f; }
  __device__ static float f(float x, float y) { return x + y; }
};
template <>
struct R<BLDP_OP_MAX> {
  __device__ static constexpr float id() { return -INFINITY; }
  __device__ static float f(float x, float y) { return __builtin_elementwise_maximum(x, y); }
};
template <>
struct R<BLDP_OP_MIN> {
  __device__ static constexpr float id() { return INFINITY; }
  __device__ static float f(float x, float y) { return __builtin_elementwise_minimum(x, y); }
};

template <int OP>
__device__ __forceinline__ float4 f4(float4 a, float4 b) {
  return make_float4(R<OP>::f(a.x, b.x), R<OP>::f(a.y, b.y), R<OP>::f(a.z, b.z),
                     R<OP>::f(a.w, b.w));
}
template <int OP>
__device__ __forceinline__ float fold4(float4 v) {
  return R<OP>::f(R<OP>::f(v.x, v.y), R<OP>::f(v.z, v.w));
}

// The lane folds of the reduce kernels run on DPP row permutes and gfx950's
// v_permlane16/32_swap (VALU only), not __shfl_xor (a ds_bpermute, an LDS round
// trip per step): profiles/r03/ab_t1v_r03a_dpp.json.
template <int CTRL>
__device__ __forceinline__ float dpp(float x) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), CTRL,
                                                              0xF, 0xF, false));
}
// Fold of op over aligned groups of W lanes (W a power of two <= 64); every
// lane of a group ends with the group's result.  An xor butterfly with the
// partners in ascending order (1, 2, 4, ...): the 4- and 8-apart steps take
// the half-mirror / mirror of a 16-lane row, which after the smaller steps
// holds exactly what the xor partner holds (every lane of an aligned block of
// 4 (8) lanes holds the same value by then); 16 and 32 apart are the gfx950
// half-swaps.  Every step is op(own, partner) on identical operands in both
// lanes, so the result is the same on every lane of the group.
template <int OP, int W>
__device__ __forceinline__ float lanes_fold(float s) {
  if constexpr (W >= 2) s = R<OP>::f(s, dpp<0xB1>(s));   // quad_perm [1,0,3,2]
  if constexpr (W >= 4) s = R<OP>::f(s, dpp<0x4E>(s));   // quad_perm [2,3,0,1]
  if constexpr (W >= 8) s = R<OP>::f(s, dpp<0x141>(s));  // row_half_mirror
  if constexpr (W >= 16) s = R<OP>::f(s, dpp<0x140>(s)); // row_mirror
  if constexpr (W >= 32) {
    const unsigned u = __builtin_bit_cast(unsigned, s);
    const auto p = __builtin_amdgcn_permlane16_swap(u, u, false, false);
    s = R<OP>::f(__builtin_bit_cast(float, (unsigned)p[0]), __builtin_bit_cast(float, (unsigned)p[1]));
  }
  if constexpr (W >= 64) {
    const unsigned u = __builtin_bit_cast(unsigned, s);
    const auto p = __builtin_amdgcn_permlane32_swap(u, u, false, false);
    s = R<OP>::f(__builtin_bit_cast(float, (unsigned)p[0]), __builtin_bit_cast(float, (unsigned)p[1]));
  }
  return s;
}
// Code-shape constants (each measured against its alternatives with
// tools/ab_variants.py, whose text-patch variants rebuild the others):
//   streaming loads carry the non-temporal hint (the window is read once):
//     +10% on cfg3 (6.35 -> 6.98 TB/s);
//   kBatch  independent 16-byte loads a lane issues before the first use
//     (4: neutral, 16: -1 .. -19%).
constexpr int kBatch = 8;
// 16-byte output stores carry the nt hint (+5% on cfg3 F=1, 5.90 -> 6.21 TB/s).
__device__ __forceinline__ void st4(float *p, float4 r) {
  const f4v v = {r.x, r.y, r.z, r.w};
  __builtin_nontemporal_store(v, reinterpret_cast<f4v *>(p));
}
// One-float-per-lane output stores: st1<1> (the row, interleaved and
// short-time-block kernels) carries the nt hint (written once, never re-read
// here; profiles/r02/ab_nt_scalar_stores.json: c0=2 F=8 +3.9%, c0=3 F=64
// +2.7%, cfg3 F=64 +1.8%, cfg2 +1.6%, cfg3 F=1024 +0.5%); st1<> (the tile,
// lane and scalar paths, which lost up to 1.9% with it) is a plain store.
template <int NT = 0>
__device__ __forceinline__ void st1(float *p, float v) {
  if constexpr (NT)
    __builtin_nontemporal_store(v, p);
  else
    *p = v;
}
// The row, interleaved and short-time-block row kernels choose per launch
// (a.st_plain, plan option "st_plain"): launches of < 2 GB keep their output
// stores plain, larger ones non-temporal.  On one box plain stores were 4-9%
// faster on the 0002 products (cfg1 -6%, cfg2 -6%, fqavby 4..16 without time
// integration -4..6%, fqavby 512..4096 at T <= 3 -3..9%) and nt stores 1-10%
// faster on the 0001 (14.4 GB) and 0000 (32 GiB) bands (profiles/r04/
// ab_*_stores_r04ad.json); on another the size rule and nt everywhere were
// even (geomean 0.994-1.002, ab_*_stplain_r04ae.json).  (The lane kernels keep
// theirs non-temporal: plain lost 2-8% there at every size.)
__device__ __forceinline__ void st1o(float *p, float v, int32_t plain) {
  if (plain)
    *p = v;
  else
    __builtin_nontemporal_store(v, p);
}
__device__ __forceinline__ void st4o(float *p, float4 r, int32_t plain) {
  const f4v v = {r.x, r.y, r.z, r.w};
  if (plain)
    *reinterpret_cast<f4v *>(p) = v;
  else
    __builtin_nontemporal_store(v, reinterpret_cast<f4v *>(p));
}
// independent float4 accumulators per lane
constexpr int kNacc = 8;
// Resident-wave caps (amdgpu_waves_per_eu) per SIMD: fewer concurrent row
// streams per CU are faster on these kernels (profiles/r01_ab_row.json,
// r02/ab_row_tpb.json, r01_ab_tilecap.json); k_reduce_row / k_reduce_rows,
// k_reduce_rowt, k_reduce_tile.
constexpr int kRowMaxWaves = 4, kRowtMaxWaves = 6, kTileMaxWaves = 3;
// Dynamic LDS per workgroup as a cap on the workgroups resident per CU (160
// KiB of LDS per CU), as kIlShm does for the interleaved kernel.  Measured
// for these kernels in round 5 and not taken (0 = no cap): the row kernels
// at 1 / 2 / 4 per CU lost 14-150% on the 0002 file and band
// (profiles/r05/ab_occ_r05d.json); the rowt kernel at 4 per CU gained 3-4%
// on the 0002 band at T <= 2 but lost 8-11% on one 0002 file and up to 3% on
// the 0001 band (ab_rowt_r05g2.json, ab_t1_0001_r05g2.json); the vector
// kernel at 2 per CU lost 60% on the 0001 band at F = 64.
constexpr unsigned kRowShm = 0, kRowtShm = 0, kVecShm = 0;
// k_reduce_narrow (F = 1, 2: a lane's float4 column down the time block,
// 16 rows in flight), 0 = no cap: at 2 / 3 / 4 workgroups per CU it was
// +2.5-7% / +-0.5% / +-0.8% on the 0000 band at F = 1, 2 and T = 8, 16
// (round 5, profiles/r05/ab_narrow_r05q.json; 14 waves per CU, half the
// cycles parked on loads: cfg3f1_sq_summary_r05p.json).
constexpr unsigned kNarrowShm = 0;
// The per-XCD contiguous tile order (xcd_order below; RedArgs::xcd_lg): the
// dispatcher sends workgroup x of a launch to XCD x % 8 on an MI355X in SPX
// mode, so in launch order every XCD streams every eighth tile, from 8
// places in each row; in the per-XCD order XCD k takes the k-th contiguous
// eighth of the tiles.  One rule, xcd_order_pays (plan_reduce), says where it
// pays; the round 5 A/B on MI355X it rests on (ratios of time, order on /
// dispatcher order; profiles/r05/ab_*xcd*.json, boxes within +-1.5% of a
// rebuilt identical library):
//   k_reduce_il, tiles of >= kIlXcdMinT rows at most kIlXcdMaxPitch apart:
//     T = 8, 16 on 16-128 MiB rows 0.91-0.97 (ab_ilxcd_r05ae.json,
//     ab_ilsmall_r05ad.json); the 0000 product's 256 MiB rows (cfg3)
//     1.005-1.022, so the pitch bound; T = 1, 2, 4 1.00-1.08, so the depth
//     bound;
//   k_reduce_row / rows (tpb = 1), rows at least kRowXcdMinPitch apart, T >= 8:
//     16 MiB rows at F = 64 / 256 0.77 / 0.76, but 256 KiB rows (the 0002 band)
//     1.03 and 2 KiB rows (the 0001 band) 1.02 (ab_rowxcd_r05ag.json);
//   k_reduce_rowt (tpb > 1), launches >= kRowtXcdBytes, rows >= kRowXcdMinPitch
//     apart: the 0000 band at T = 1, 2 0.95-0.97; smaller launches mixed, one
//     0002 file 1.07-1.13 (ab_rowtxcd_r05an.json, ab_rowtxcd_gate_r05ao.json);
//   k_reduce_narrowt at F = 2 on launches >= kRowtXcdBytes: the 0000 band at
//     T = 1 / 2 / 4 0.93 / 0.96 / 0.94; F = 1 mixed, and the 0002 band at F = 2
//     T = 1 lost 4% on a second box (ab_narrowtxcd_r05ar.json, _r05as.json,
//     ab_narrowtxcd_confirm_r05at.json);
//   k_reduce_narrow, k_reduce_vec: always (the 0000 band at F = 1, 2
//     0.975-0.987, ab_narrowxcd_r05am.json; the 0001 band at F = 64 T = 16
//     0.963, cfg4 0.992, ab_vecxcd_r05ak.json);
//   k_reduce_tile 0.94-1.035 by shape, k_reduce_wavet 1.03-1.045
//     (ab_tilexcd_r05ar.json, ab_wavetxcd_r05aw.json), and the kurtosis and
//     typed kernels (ab_kregsxcd_r05ai, ab_kmidxcd_r05ah, ab_kleafxcd_r05am,
//     ab_typedxcd_r05an: 0.97-1.08): never (round 6: their branches removed;
//     tools/ab_variants.py re-creates the reduce ones by patching the rule).
// Only on a device whose XCD count is a power of two (hipDeviceAttribute-
// NumberOfXccs: 8 in SPX mode, 4 / 2 / 1 in the DPX / QPX / CPX partitions,
// where the order spreads over that many XCDs; the bounds were measured in SPX).
constexpr int kIlXcdMinT = 8;
constexpr int64_t kRowXcdMinPitch = (int64_t)4 << 20;
constexpr int64_t kIlXcdMaxPitch = (int64_t)128 << 20;
constexpr int64_t kRowtXcdBytes = (int64_t)1 << 30;

// Workgroup x of a launch of X in the per-XCD contiguous order over 2^lg
// XCDs: x runs on XCD x % 2^lg and takes tile (x % 2^lg) * (X / 2^lg) +
// x / 2^lg.  lg = 0 (the plan's "no"), or a grid 2^lg does not divide: x.
__device__ __forceinline__ uint32_t xcd_order(uint32_t x, uint32_t X, int lg) {
  const uint32_t m = (1u << lg) - 1u;
  if (lg == 0 || (X & m)) return x;
  return (x & m) * (X >> lg) + (x >> lg);
}

// The short-time-block kernels (k_reduce_rowt, k_reduce_narrowt,
// k_reduce_lanet) also take tavby = 3 and 8, not only 1, 2, 4 (plan option
// "t38"; the 512-channel 0001 product at tavby = 3 ran one 3-row block per
// wave with half the waves idle: 2.4-2.7 TB/s).  narrowt: fqavby = 2 at
// tavby = 3 only (fqavby = 1 lost 7% on the 0002 band; at tavby = 8
// narrow_tile's one full batch sums in another order).
// profiles/r03/ab_t38_r03t.json
#define BLDP_T38_CASES(M, X) case 3: M(X, 3) case 8: M(X, 8)

// Pairwise fold of the per-lane accumulators into acc[0].
template <int OP>
__device__ __forceinline__ float4 fold_acc(float4 (&acc)[kNacc]) {
#pragma unroll
  for (int w = kNacc / 2; w >= 1; w /= 2)
#pragma unroll
    for (int q = 0; q < w; ++q) acc[q] = f4<OP>(acc[q], acc[q + w]);
  return acc[0];
}
__device__ __forceinline__ float4 ld4(const float *p) {
  const f4u v = __builtin_nontemporal_load(reinterpret_cast<const f4u *>(p));
  return make_float4(v.x, v.y, v.z, v.w);
}
// Groups of 3 float4 per lane on the vector path (fqavby = 12, 24, 48, ...,
// 768) have a compiled K4 = 3 form with plain loads: an nt load covers a third
// of each line at the 48-byte lane pitch and the next instruction re-reads it
// from HBM (profiles/r03/ab_k3_r03n.json: generic loop 10.97, nt 7.43, plain
// 5.55 ms on the 0000 band at F = 12).
template <bool PLAIN>
__device__ __forceinline__ float4 ld4x(const float *p) {
  if constexpr (PLAIN) {
    const f4u v = *reinterpret_cast<const f4u *>(p);
    return make_float4(v.x, v.y, v.z, v.w);
  } else {
    return ld4(p);
  }
}
// The rows of a block left after the last full batch (all of them when T is
// below the batch size: tavby = 3, 8, 9, ...), loaded together and then
// chained into the first accumulator in row order: the same sums as one row
// at a time, with up to N - 1 loads in flight per lane instead of one
// (profiles/r03/ab_row_tail_r03l.json: +11 .. +48%).
template <int OP, int N, bool PLAIN = false>
__device__ __forceinline__ float4 tail_rows(float4 acc, const float *p, int64_t st, int64_t nrows) {
  static_assert(N <= 16, "tail_rows: at most 15 rows");
  // nrows (< N, wave-uniform) as 8 + 4 + 2 + 1 rows: every load issued before
  // the first add, no predicated array elements
  float4 v8[8], v4[4], v2[2], v1;
  const bool b8 = N > 8 && (nrows & 8), b4 = N > 4 && (nrows & 4), b2 = N > 2 && (nrows & 2),
             b1 = nrows & 1;
  const float *q = p;
  if (b8) {
#pragma unroll
    for (int u = 0; u < 8; ++u) v8[u] = ld4x<PLAIN>(q + u * st);
    q += 8 * st;
  }
  if (b4) {
#pragma unroll
    for (int u = 0; u < 4; ++u) v4[u] = ld4x<PLAIN>(q + u * st);
    q += 4 * st;
  }
  if (b2) {
#pragma unroll
    for (int u = 0; u < 2; ++u) v2[u] = ld4x<PLAIN>(q + u * st);
    q += 2 * st;
  }
  if (b1) v1 = ld4x<PLAIN>(q);
  if (b8) {
#pragma unroll
    for (int u = 0; u < 8; ++u) acc = f4<OP>(acc, v8[u]);
  }
  if (b4) {
#pragma unroll
    for (int u = 0; u < 4; ++u) acc = f4<OP>(acc, v4[u]);
  }
  if (b2) {
#pragma unroll
    for (int u = 0; u < 2; ++u) acc = f4<OP>(acc, v2[u]);
  }
  if (b1) acc = f4<OP>(acc, v1);
  return acc;
}

// blockIdx.x -> (bc, i, chunk, to, bank); bc fastest so that consecutive
// workgroups stream consecutive channel segments of one row.
struct Coord {
  int64_t bc, i, chunk, to;
  int bank;
};
__device__ __forceinline__ Coord decompose(const RedArgs &a, int64_t tile) {
  Coord c;
  int64_t b = tile;
  c.bc = b % a.blocks_c;
  b /= a.blocks_c;
  c.i = b % a.ni;
  b /= a.ni;
  c.chunk = b % a.nchunk;
  b /= a.nchunk;
  c.to = b % a.nto;
  c.bank = (int)(b / a.nto);
  return c;
}

template <int OP>
__device__ __forceinline__ float finish(float s, const RedArgs &a) {
  if (OP == BLDP_OP_MEAN) return s / a.div;
  return s;
}

// ---------------------------------------------------------------------------
// Vector path, F % 4 == 0.  A group of F channels (G4 = F/4 float4 per row)
// is owned by LPG lanes (largest power of two dividing G4, <= 64); each lane
// reads K4 = G4/LPG float4 per row.  A wave therefore owns 64/LPG consecutive
// outputs and every load instruction covers LPG*16 contiguous bytes per group
// (1 KiB per wave when K4 == 1 or LPG == 64).  `ts` waves split the T rows of
// a tile; 4/ts tiles per workgroup.
template <int OP, int LPG, int K4C>
__device__ __forceinline__ void vec_tile(const RedArgs &a, int64_t tile) {
  constexpr int OPW = 64 / LPG;
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int ts = a.ts;
  const int wt = wave / ts;
  const int tsi = wave - wt * ts;
  const Coord c = decompose(a, tile);
  const int g = lane / LPG, j = lane % LPG;
  const int64_t co = (c.bc * (4 / ts) + wt) * OPW + g;
  const bool valid = co < a.nco;
  const int64_t r0 = c.chunk * a.rows_per_chunk;
  const int64_t r1 = min(a.T, r0 + a.rows_per_chunk);
  const float id = R<OP>::id();

  float4 acc[kNacc];
#pragma unroll
  for (int q = 0; q < kNacc; ++q) acc[q] = make_float4(id, id, id, id);

  if (valid) {
    const float *p = a.in[c.bank] + a.in_off + c.i * a.in_ld_i +
                     (c.to * a.T + r0 + tsi) * a.in_ld_t + co * a.F + 4 * j;
    int64_t nrows = r1 - r0 - tsi;
    nrows = nrows > 0 ? (nrows + ts - 1) / ts : 0;
    const int64_t rstep = (int64_t)ts * a.in_ld_t;
    if constexpr (K4C > 0) {
      constexpr int RB = (K4C >= kBatch) ? 1 : kBatch / K4C;
      constexpr int NV = RB * K4C;
      constexpr bool PL = K4C == 3;
      for (; nrows >= RB; nrows -= RB) {
        float4 v[NV];
#pragma unroll
        for (int u = 0; u < RB; ++u)
#pragma unroll
          for (int k = 0; k < K4C; ++k) v[u * K4C + k] = ld4x<PL>(p + u * rstep + 4 * k * LPG);
        p += RB * rstep;
#pragma unroll
        for (int q = 0; q < NV; ++q) acc[q % kNacc] = f4<OP>(acc[q % kNacc], v[q]);
      }
      if constexpr (RB > 1 && K4C <= kNacc) {
        // the last rows (< RB) together; column k's rows go to accumulator k
        // alone, in row order, as in the loop below
#pragma unroll
        for (int k = 0; k < K4C; ++k)
          acc[k] = tail_rows<OP, RB, PL>(acc[k], p + 4 * k * LPG, rstep, nrows);
        nrows = 0;
      }
      for (; nrows > 0; --nrows) {
#pragma unroll
        for (int k = 0; k < K4C; ++k)
          acc[k % kNacc] = f4<OP>(acc[k % kNacc], ld4x<PL>(p + 4 * k * LPG));
        p += rstep;
      }
    } else {
      const int K4 = a.k4;
      for (; nrows > 0; --nrows) {
        int k = 0;
        for (; k + 8 <= K4; k += 8) {
          float4 v[8];
#pragma unroll
          for (int u = 0; u < 8; ++u) v[u] = ld4(p + 4 * (k + u) * LPG);
#pragma unroll
          for (int u = 0; u < 8; ++u) acc[u % kNacc] = f4<OP>(acc[u % kNacc], v[u]);
        }
        for (; k < K4; ++k) acc[0] = f4<OP>(acc[0], ld4(p + 4 * k * LPG));
        p += rstep;
      }
    }
  }
  float s = fold4<OP>(fold_acc<OP>(acc));

  // combine the LPG lanes of a group (xor butterfly inside aligned segments)
  s = lanes_fold<OP, LPG>(s);

  if (ts > 1) {  // combine the waves that split the time rows, through LDS
    __shared__ float red[4][64];
    red[wave][lane] = s;
    __syncthreads();
    if (tsi == 0)
      for (int q = 1; q < ts; ++q) s = R<OP>::f(s, red[wave + q][lane]);
    __syncthreads();  // red[] is reused by the next tile of a grid-stride loop
  }
  if (tsi == 0 && j == 0 && valid) {
    if (a.nchunk == 1) {
      st1(a.out + c.bank * a.out_bank + c.i * a.out_ld_i + c.to * a.out_ld_t + co, finish<OP>(s, a));
    } else {
      a.ws[(((c.chunk * a.nbank + c.bank) * a.nto + c.to) * a.ni + c.i) * a.nco + co] = s;
    }
  }
}

// ---------------------------------------------------------------------------
// Narrow path, F in {1, 2}: one float4 (4 channels) per lane per row; no
// cross-lane work.  F == 1 is pure time integration (gather-stress variant).
template <int OP, int F>
__device__ __forceinline__ void narrow_tile(const RedArgs &a, int64_t tile) {
  const Coord c = decompose(a, tile);
  const int64_t q4 = c.bc * kBlock + threadIdx.x;  // float4 column
  const int64_t nc4 = a.nco * F / 4;
  if (q4 >= nc4) return;
  const int64_t r0 = c.chunk * a.rows_per_chunk;
  const int64_t r1 = min(a.T, r0 + a.rows_per_chunk);
  const float id = R<OP>::id();
  float4 acc[kNacc];
#pragma unroll
  for (int q = 0; q < kNacc; ++q) acc[q] = make_float4(id, id, id, id);
  const float *p =
      a.in[c.bank] + a.in_off + c.i * a.in_ld_i + (c.to * a.T + r0) * a.in_ld_t + 4 * q4;
  const int64_t st = a.in_ld_t;
  int64_t nrows = r1 - r0;
  for (; nrows >= kBatch; nrows -= kBatch) {
    float4 v[kBatch];
#pragma unroll
    for (int u = 0; u < kBatch; ++u) v[u] = ld4(p + u * st);
    p += kBatch * st;
#pragma unroll
    for (int u = 0; u < kBatch; ++u) acc[u % kNacc] = f4<OP>(acc[u % kNacc], v[u]);
  }
  acc[0] = tail_rows<OP, kBatch>(acc[0], p, st, nrows);
  float4 r = fold_acc<OP>(acc);
  const int64_t co = q4 * (4 / F);
  if (a.nchunk == 1) {
    float *o = a.out + c.bank * a.out_bank + c.i * a.out_ld_i + c.to * a.out_ld_t + co;
    if (F == 1) {
      r = make_float4(finish<OP>(r.x, a), finish<OP>(r.y, a), finish<OP>(r.z, a),
                      finish<OP>(r.w, a));
      if (a.vec_out) {
        st4(o, r);
      } else {
        o[0] = r.x; o[1] = r.y; o[2] = r.z; o[3] = r.w;
      }
    } else {
      const float x = finish<OP>(R<OP>::f(r.x, r.y), a), y = finish<OP>(R<OP>::f(r.z, r.w), a);
      if (a.vec_out) {
        *reinterpret_cast<float2 *>(o) = make_float2(x, y);
      } else {
        o[0] = x; o[1] = y;
      }
    }
  } else {
    float *o = a.ws + (((c.chunk * a.nbank + c.bank) * a.nto + c.to) * a.ni + c.i) * a.nco + co;
    if (F == 1) {
      *reinterpret_cast<float4 *>(o) = r;
    } else {
      *reinterpret_cast<float2 *>(o) = make_float2(R<OP>::f(r.x, r.y), R<OP>::f(r.z, r.w));
    }
  }
}

// The narrow path for short time blocks (T = 1, 2, 4; e.g. fqavby = 2 with
// the reference's own fqav, no time integration), organised like
// k_reduce_rowt: 16 / T time blocks per workgroup, 2 or 4 time groups per
// workgroup for windows of <= 128 float4 columns.  Each block is summed and
// stored exactly as narrow_tile does it (bit-identical).  No resident-wave cap
// (the narrow kernels run uncapped: a cap of 4 cost k_reduce_narrow 1.2%).
// Plan option "narrow_tpb": 2 (default) = use it for T in {1, 2, 4}, the copy
// (fqavby = tavby = 1) included; 1 = not for the copy; 0 = k_reduce_narrow.
template <int OP, int F, int T, int NRW>
__global__ __launch_bounds__(kBlock) void k_reduce_narrowt(const RedArgs a) {
  constexpr int TPB = NRW / T, NR = TPB * T;
  const int tid = threadIdx.x;
  const uint32_t bx = xcd_order(blockIdx.x, gridDim.x, a.xcd_lg);
  const uint32_t bc = (uint32_t)a.blocks_c;
  const int sh = a.tsub_log2, cw = kBlock >> sh;
  const uint32_t tq = bx / bc, i = blockIdx.y;
  const int64_t tg = ((int64_t)tq << sh) + (tid >> (8 - sh));
  const int bank = blockIdx.z;
  const int64_t q4 = (int64_t)(bx - tq * bc) * kBlock + (tid & (cw - 1));  // float4 column
  const int64_t to0 = tg * TPB;
  if (q4 >= a.nco * F / 4 || to0 >= a.nto) return;  // (no cross-lane work below)
  const int nb = (int)min((int64_t)TPB, a.nto - to0);
  const float id = R<OP>::id();
  const float4 id4 = make_float4(id, id, id, id);
  const float *p = a.in[bank] + a.in_off + (int64_t)i * a.in_ld_i + to0 * T * a.in_ld_t + 4 * q4;
  const int64_t ld = a.in_ld_t;
  float4 v[NR];
#pragma unroll
  for (int u = 0; u < NR; ++u)
    if (u < nb * T) v[u] = ld4(p + u * ld);
  const int64_t co = q4 * (4 / F);
#pragma unroll
  for (int b = 0; b < TPB; ++b) {
    if (b < nb) {
      // narrow_tile's accumulators for T < kBatch rows: chained into the
      // first, then its fold with the identities = one op with the identity
      float4 r = id4;
#pragma unroll
      for (int u = 0; u < T; ++u) r = f4<OP>(r, v[b * T + u]);
      if constexpr (kNacc > 1) r = f4<OP>(r, id4);
      float *o = a.out + bank * a.out_bank + (int64_t)i * a.out_ld_i + (to0 + b) * a.out_ld_t + co;
      if (F == 1) {
        r = make_float4(finish<OP>(r.x, a), finish<OP>(r.y, a), finish<OP>(r.z, a),
                        finish<OP>(r.w, a));
        if (a.vec_out) {
          st4(o, r);
        } else {
          o[0] = r.x; o[1] = r.y; o[2] = r.z; o[3] = r.w;
        }
      } else {
        const float x = finish<OP>(R<OP>::f(r.x, r.y), a), y = finish<OP>(R<OP>::f(r.z, r.w), a);
        if (a.vec_out) {
          *reinterpret_cast<float2 *>(o) = make_float2(x, y);
        } else {
          o[0] = x; o[1] = y;
        }
      }
    }
  }
}

// ---------------------------------------------------------------------------
// Narrow path for windows that start off a 16-byte boundary (unit channel
// step, F = 1, e.g. idxs = (2:n, :, :) with time integration; F = 2 with
// plan option narrow_mis = 2).  Each wave owns 256 window channels = 64 output float4
// (1 KiB of output, aligned like the output row).  Lane L streams the ALIGNED
// input float4 column L (lane 63 also column 64) and sums its T rows in
// registers exactly like narrow_tile; output float4 L is then elements
// mis..3 of column L and 0..mis-1 of column L+1, taken from the next lane by
// shuffle.  No LDS, no barrier; the input read is the window plus one float4
// per wave.
constexpr int kMisSpan = 4 * 256;  // window channels per workgroup (4 waves x 256)
template <int OP, int F>
__device__ __forceinline__ void narrow_mis_tile(const RedArgs &a, int64_t tile) {
  const Coord c = decompose(a, tile);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t nwin = a.nco * F;  // window channels
  const int64_t x0 = c.bc * kMisSpan + wave * 256;
  if (x0 >= nwin) return;  // a wave past the window's end (no barrier follows)
  const int64_t abs0 = a.in_off + c.i * a.in_ld_i + x0;
  const int mis = (int)(abs0 & 3);  // bank pointers and row pitches are 16-byte aligned
  const int cnt = (int)min<int64_t>(256, nwin - x0);
  const int ncol = (mis + cnt + 3) >> 2;  // <= 65
  const bool extra = lane == 63 && ncol > 64;
  const int64_t r0 = c.chunk * a.rows_per_chunk;
  const int64_t r1 = min(a.T, r0 + a.rows_per_chunk);
  const float id = R<OP>::id();
  float4 acc[kNacc], ax = make_float4(id, id, id, id);
#pragma unroll
  for (int q = 0; q < kNacc; ++q) acc[q] = ax;
  if (lane < ncol) {
    const float *p = a.in[c.bank] + (abs0 - mis) + (c.to * a.T + r0) * a.in_ld_t + 4 * lane;
    const int64_t st = a.in_ld_t;
    int64_t nrows = r1 - r0;
    for (; nrows >= kBatch; nrows -= kBatch) {
      float4 v[kBatch], w[kBatch];
#pragma unroll
      for (int u = 0; u < kBatch; ++u) v[u] = ld4(p + u * st);
      if (extra) {
#pragma unroll
        for (int u = 0; u < kBatch; ++u) w[u] = ld4(p + 4 + u * st);
#pragma unroll
        for (int u = 0; u < kBatch; ++u) ax = f4<OP>(ax, w[u]);
      }
      p += kBatch * st;
#pragma unroll
      for (int u = 0; u < kBatch; ++u) acc[u % kNacc] = f4<OP>(acc[u % kNacc], v[u]);
    }
    acc[0] = tail_rows<OP, kBatch>(acc[0], p, st, nrows);
    if (extra) ax = tail_rows<OP, kBatch>(ax, p + 4, st, nrows);
  }
  const float4 lo = fold_acc<OP>(acc);
  float4 hi = make_float4(__shfl_down(lo.x, 1, 64), __shfl_down(lo.y, 1, 64),
                          __shfl_down(lo.z, 1, 64), __shfl_down(lo.w, 1, 64));
  if (lane == 63) hi = ax;
  const int nv = min(4, cnt - 4 * lane);  // window channels of this lane's output float4
  if (nv <= 0) return;
  float4 r;
  switch (mis) {
    case 1: r = make_float4(lo.y, lo.z, lo.w, hi.x); break;
    case 2: r = make_float4(lo.z, lo.w, hi.x, hi.y); break;
    case 3: r = make_float4(lo.w, hi.x, hi.y, hi.z); break;
    default: r = lo;
  }
  const int64_t co = (x0 + 4 * lane) / F;  // first output of this lane (x0 is even)
  float o[4] = {r.x, r.y, r.z, r.w};
  int no = nv;
  if (F == 2) {
    o[0] = R<OP>::f(r.x, r.y);
    o[1] = R<OP>::f(r.z, r.w);
    no = nv / 2;
  }
  float *dst;
  if (a.nchunk == 1) {
    dst = a.out + c.bank * a.out_bank + c.i * a.out_ld_i + c.to * a.out_ld_t + co;
#pragma unroll
    for (int q = 0; q < 4; ++q) o[q] = finish<OP>(o[q], a);
  } else {
    dst = a.ws + (((c.chunk * a.nbank + c.bank) * a.nto + c.to) * a.ni + c.i) * a.nco + co;
  }
  if (F == 1 && no == 4 && a.nchunk == 1 && a.vec_out) {
    st4(dst, make_float4(o[0], o[1], o[2], o[3]));
  } else if (F == 2 && no == 2 && (a.nchunk > 1 || a.vec_out)) {  // (ws: dense, even co)
    *reinterpret_cast<float2 *>(dst) = make_float2(o[0], o[1]);
  } else {
#pragma unroll
    for (int q = 0; q < 4; ++q)
      if (q < no) dst[q] = o[q];
  }
}

// ---------------------------------------------------------------------------
// Lane path (PATH_LANE): unit channel step, small F that is not a multiple of
// 4 (2, 3, 5, 6, 7), any dword alignment (odd F, or F = 2 off a 16-byte
// boundary).  One lane per output group: its F channels of a row are adjacent
// floats, which the compiler issues as one dwordx{2,3} (F = 2, 3) or
// dwordx4 + dwordx{1,2,3} (F = 5..7) load, so a wave-instruction streams 64*F*4
// contiguous bytes with no LDS and no cross-lane work; 8 rows in flight, two
// accumulator sets.  A/B against the tile path's LDS fold (8 banks x 2^26
// channels x 16 spectra, profiles/r02/ab_lane.json, ab_cluster.json): F = 3
// 6.69 vs 6.74 ms on one box but 5.78 vs 5.57 on another, F = 2 (c0 = 1) 6.85
// vs 6.92, F = 5 10.4 vs 6.5 and F = 7 7.8 vs 6.4 (a dwordx4 + dwordx{1,3}
// pair per lane at a 20- / 28-byte lane pitch splits every wave-instruction
// into many partial lines).  A third form, float4 columns in clusters of F
// lanes gathered by shuffles, lost to both (F = 3 6.18, F = 7 5.77 ms: its
// one-float stores are scattered over 4 instructions).  So (plan options):
//   lane   1 (default) = F in {2, 3, 5, 6, 7} only where the tile path cannot
//          run (row pitches that are not multiples of 4 floats; the
//          alternative is the scalar path); 2 = always; 0 = off
//   lane3  1 (default) = F = 3 on the lane kernel everywhere: one dwordx3 per
//          lane covers whole lines, and on narrow windows (the 512-channel
//          0001 product, 170 groups a row) the tile path ran at 2.8-4.3 TB/s
//          against the lane kernel's 1.6x more
//          (profiles/r03/ab_grid1_lane2_r03v.json)
template <int OP, int F>
__device__ __forceinline__ void lane_tile(const RedArgs &a, int64_t tile) {
  const Coord c = decompose(a, tile);
  const int64_t co = c.bc * kBlock + threadIdx.x;
  if (co >= a.nco) return;
  const int64_t r0 = c.chunk * a.rows_per_chunk;
  const int64_t r1 = min(a.T, r0 + a.rows_per_chunk);
  const float id = R<OP>::id();
  float acc[2][F];
#pragma unroll
  for (int q = 0; q < 2; ++q)
#pragma unroll
    for (int f = 0; f < F; ++f) acc[q][f] = id;
  const float *p =
      a.in[c.bank] + a.in_off + c.i * a.in_ld_i + (c.to * a.T + r0) * a.in_ld_t + co * F;
  const int64_t st = a.in_ld_t;
  int64_t nrows = r1 - r0;
  for (; nrows >= kBatch; nrows -= kBatch) {
    float v[kBatch][F];
#pragma unroll
    for (int u = 0; u < kBatch; ++u)
#pragma unroll
      for (int f = 0; f < F; ++f) v[u][f] = __builtin_nontemporal_load(p + u * st + f);
    p += kBatch * st;
#pragma unroll
    for (int u = 0; u < kBatch; ++u)
#pragma unroll
      for (int f = 0; f < F; ++f) acc[u & 1][f] = R<OP>::f(acc[u & 1][f], v[u][f]);
  }
  for (; nrows > 0; --nrows) {
#pragma unroll
    for (int f = 0; f < F; ++f) acc[0][f] = R<OP>::f(acc[0][f], __builtin_nontemporal_load(p + f));
    p += st;
  }
  float s = R<OP>::f(acc[0][0], acc[1][0]);
#pragma unroll
  for (int f = 1; f < F; ++f) s = R<OP>::f(s, R<OP>::f(acc[0][f], acc[1][f]));
  if (a.nchunk == 1)
    st1(a.out + c.bank * a.out_bank + c.i * a.out_ld_i + c.to * a.out_ld_t + co, finish<OP>(s, a));
  else
    a.ws[(((c.chunk * a.nbank + c.bank) * a.nto + c.to) * a.ni + c.i) * a.nco + co] = s;
}

// The lane path for short time blocks (T = 1, 2, 4; T = 1 is the reference's
// own fqav with no time integration) and small groups that are not a power of
// two: F = 3, 5, 6, 7, 12 (e.g. fqavby = 3 or 12 on a 65535- / 65532-channel
// window of a 0002 product).  One lane per output group as in lane_tile, but a
// workgroup takes TPB = NRW / T consecutive time blocks of its 256 groups, so
// NRW rows (F * NRW <= 48 floats) are in flight per lane and every workgroup
// streams NRW x 1 KiB..3 KiB of rows instead of a single row segment (the tile
// path's one-row workgroups at T = 1: 0.44 of the read/write-mix ceiling on the
// 0002 band at F = 3, profiles/r03/).  A row's F floats are one dwordx2 / x3 /
// x4 per lane where F <= 4 (one wave-instruction covers whole 128-byte lines:
// non-temporal), else several 16-byte pieces at an F*4-byte lane pitch, which
// each cover every line only in part: those are plain loads, so the lines the
// next piece needs are still in L1 (nt loads there read every line from HBM
// about twice, the vector path's 1.98x at F = 12).  Stores: one float per lane,
// 1 KiB per workgroup-instruction.  Measured and not taken (round 3,
// profiles/r03/ab_t1v_r03d.json): each wave staging its rows through LDS with
// coalesced float4 loads and every lane reading its group back, F = 12 0.144
// vs 0.125 ms, F = 3 0.171 vs 0.162 ms on the 0002 band (the LDS round trip
// and the workgroup barrier cost more than the partial-line loads).
// Plan option "lanet": 1 (default) = use it for T in {1, 2, 3, 4, 8}; 0 = the
// lane / tile / vector paths.  Measured forms (tools/ab_variants.py text
// patches rebuild them): F = 3 rows as one non-temporal dwordx3 (plain: slower);
// 8 rows per lane for every F (16 for F <= 3 and 4 for F > 6 were the defaults
// until the aligned output segments below, with which 8 is 10% (F = 3) and 3%
// (F = 12) faster, profiles/r03/ab_t1v_r03h.json); F > 4 pieces as plain
// loads (nt: slower); one column set per lane.  (G consecutive groups per lane
// with whole float4 loads and float4 / float2 stores was measured too,
// profiles/r03/ab_t1v_r03e.json: F = 3 with 4 groups per lane 0.297 vs 0.164
// ms, not taken.)  Each output row's 256-group segments start on a 64-byte
// boundary of the product (the segment grid shifted by that row's
// misalignment), so no two workgroups share a line and only row ends are
// partial writes.  A product row of nco groups starts on a line only when nco
// is a multiple of 16; otherwise every workgroup boundary fell inside a line
// and each of those lines went out as two partial writes from two workgroups.
// 0002 band, fqavby = 3 (21845 groups a row): 0.169 -> 0.134 ms with 8 rows
// per lane; fqavby = 12 0.125 -> 0.122 (profiles/r03/ab_t1v_r03g_oalign.json,
// bit-identical).  Plan option "lanet_pack": 1 (default) = windows of <= 113
// groups share a workgroup between 2 or 4 time groups.
constexpr int lanet_oalign_pad() { return 15; }  // output segments on 64-byte lines
typedef float f2u __attribute__((ext_vector_type(2), aligned(4)));
typedef float f2v __attribute__((ext_vector_type(2)));
typedef float f3u __attribute__((ext_vector_type(3), aligned(4)));
template <typename V>
__device__ __forceinline__ V ldv(const float *p, bool nt) {
  return nt ? __builtin_nontemporal_load(reinterpret_cast<const V *>(p))
            : *reinterpret_cast<const V *>(p);
}
template <int F>
__device__ __forceinline__ void ldF(const float *p, float (&x)[F]) {
  if constexpr (F == 3) {
    const f3u v = ldv<f3u>(p, true);  // one nt dwordx3: whole lines per wave
    x[0] = v.x; x[1] = v.y; x[2] = v.z;
  } else {
    int f = 0;
#pragma unroll
    for (; f + 4 <= F; f += 4) {
      const f4u v = ldv<f4u>(p + f, false);
      x[f] = v.x; x[f + 1] = v.y; x[f + 2] = v.z; x[f + 3] = v.w;
    }
    if constexpr (F % 4 == 3) {
      const f3u v = ldv<f3u>(p + f, false);
      x[f] = v.x; x[f + 1] = v.y; x[f + 2] = v.z;
    } else if constexpr (F % 4 == 2) {
      const f2u v = ldv<f2u>(p + f, false);
      x[f] = v.x; x[f + 1] = v.y;
    } else if constexpr (F % 4 == 1) {
      x[f] = p[f];
    }
  }
}
constexpr int kLanetRows = 8;  // rows per lane (every F)
template <int OP, int F, int T>
__global__ __launch_bounds__(kBlock) void k_reduce_lanet(const RedArgs a) {
  constexpr int TPB = kLanetRows / T, NRW = TPB * T;  // (T = 3: 6 rows)
  static_assert(TPB >= 1, "k_reduce_lanet: rows per lane");
  const int tid = threadIdx.x;
  const uint32_t bx = blockIdx.x, bc = (uint32_t)a.blocks_c;
  const uint32_t tq = bx / bc, i = blockIdx.y;
  const int bank = blockIdx.z;
  const float id = R<OP>::id();
  const int64_t ld = a.in_ld_t;
  // narrow windows (nco + 15 <= 128 / 64 groups): 2 / 4 time groups share the
  // workgroup, 256 >> sh lanes each (a.tsub_log2 = sh; 0 otherwise)
  const int sh = a.tsub_log2, cw = kBlock >> sh, lt = tid & (cw - 1);
  const int64_t tp0 = (((int64_t)tq << sh) + (tid >> (8 - sh))) * TPB;  // first time block
  const int nbp = (int)max((int64_t)0, min((int64_t)TPB, a.nto - tp0));
  // per output row b: this lane's group, shifted so the workgroup's outputs
  // of that row start on a 64-byte line of the product
  float *orow[TPB];
  int64_t g[TPB];
  bool ok[TPB];
  const int64_t cb = (int64_t)(bx - tq * bc) * cw;
#pragma unroll
  for (int b = 0; b < TPB; ++b) {
    orow[b] = a.out + bank * a.out_bank + (int64_t)i * a.out_ld_i + (tp0 + b) * a.out_ld_t;
    const int64_t s = (int64_t)((reinterpret_cast<uintptr_t>(orow[b]) >> 2) & 15);
    g[b] = cb - s + lt;
    ok[b] = b < nbp && g[b] >= 0 && g[b] < a.nco;
  }
  float v[NRW][F];
  const float *p = a.in[bank] + a.in_off + (int64_t)i * a.in_ld_i + tp0 * T * ld;
#pragma unroll
  for (int u = 0; u < NRW; ++u) {
    if (ok[u / T]) {
      ldF<F>(p + u * ld + g[u / T] * F, v[u]);
    } else {
#pragma unroll
      for (int f = 0; f < F; ++f) v[u][f] = id;
    }
  }
#pragma unroll
  for (int b = 0; b < TPB; ++b) {
    // a block's F x T values in the reference's order: the F channels of a
    // spectrum in sequence (fqav's sum over dims = 1), spectrum after spectrum
    float acc = id;
#pragma unroll
    for (int r = 0; r < T; ++r)
#pragma unroll
      for (int f = 0; f < F; ++f) acc = R<OP>::f(acc, v[b * T + r][f]);
    if (ok[b]) st1<1>(orow[b] + g[b], finish<OP>(acc, a));
  }
}

// k_reduce_lanet over a stitched band of narrow banks (the 0001 band at
// fqavby = 3 / 12: 170 / 42 groups a bank row): the lanes run along the
// stitched product row, lane k of a time group taking group k % nco of bank
// k / nco, so a workgroup's outputs of each of its rows are 256 consecutive
// floats of the product (1 KiB, whole 64-byte lines where the row is
// line-aligned) instead of one bank's short segment with a partial line at
// each end, and every lane is busy (lanet left 86 of 256 idle at 170 groups).
// Rows and blocks are summed exactly as k_reduce_lanet sums them
// (bit-identical).  Plan option "lane_bpack".
template <int OP, int F, int T>
__global__ __launch_bounds__(kBlock) void k_reduce_lanes(const RedArgs a) {
  constexpr int TPB = kLanetRows / T, NRW = TPB * T;
  const uint32_t nbx = (uint32_t)a.blocks_c, bx = blockIdx.x, tq = bx / nbx, i = blockIdx.y;
  const uint32_t k = (bx - tq * nbx) * kBlock + threadIdx.x;  // position in the stitched row
  const uint32_t nco = (uint32_t)a.nco, bank = k / nco, g = k - bank * nco;
  const bool in = bank < (uint32_t)a.nbank;
  const float id = R<OP>::id();
  const int64_t ld = a.in_ld_t, tp0 = (int64_t)tq * TPB;
  const int nbp = (int)min((int64_t)TPB, a.nto - tp0);
  float v[NRW][F];
  const float *p = a.in[in ? bank : 0] + a.in_off + (int64_t)i * a.in_ld_i + tp0 * T * ld +
                   (int64_t)g * F;
#pragma unroll
  for (int u = 0; u < NRW; ++u) {
    if (in && u / T < nbp) {
      ldF<F>(p + u * ld, v[u]);
    } else {
#pragma unroll
      for (int f = 0; f < F; ++f) v[u][f] = id;
    }
  }
  float *o = a.out + (int64_t)i * a.out_ld_i + tp0 * a.out_ld_t + k;  // (out_bank == nco)
#pragma unroll
  for (int b = 0; b < TPB; ++b) {
    float acc = id;
#pragma unroll
    for (int r = 0; r < T; ++r)
#pragma unroll
      for (int f = 0; f < F; ++f) acc = R<OP>::f(acc, v[b * T + r][f]);
    if (in && b < nbp) st1<1>(o + b * a.out_ld_t, finish<OP>(acc, a));
  }
}

// fqavby = 12 with short time blocks (T = 1, 2, 3, 4, 8; e.g. the 0001 band
// without time integration, 42 groups a bank row): lanes on float4 columns,
// three to a group, so every wave-instruction reads 1 KiB contiguous, where
// k_reduce_lanet's one lane per group read three 16-byte pieces at a 48-byte
// lane pitch (three instructions touching every line).  A workgroup of three
// waves takes 64 consecutive groups of the stitched product row (bank-major:
// several narrow banks per workgroup) and TPB = 16 / T time blocks; each
// lane sums its column over a block's T rows and folds the float4, the three
// partials of a group meet in LDS, and the workgroup stores 64 consecutive
// outputs (256 bytes) per product row.  Summation order: per lane the T rows
// in sequence, then (x + y) + (z + w); the group's three lane sums left to
// right (integer data: the oracle's bits; Float32 data within the stated
// tolerance, as every path).  Plan option "col3".
constexpr int kCol3Threads = 192;
template <int OP, int T>
__global__ __launch_bounds__(kCol3Threads) void k_reduce_col3(const RedArgs a) {
  // 4 rows per lane at T <= 4: 8 rows were 2-8% faster than 16 on the 0001
  // and 0002 bands at T = 1..8 (profiles/r04/ab_t1_0001_r04o.json,
  // ab_grid_r04o.json), 4 another 6% at T = 1 and 2% at T = 3 (ab_t1v_r04v.json,
  // ab_k3_r04v.json)
  constexpr int TPB = 4 / T > 0 ? 4 / T : 1, NR = TPB * T;
  const uint32_t nbx = (uint32_t)a.blocks_c, bx = blockIdx.x, tq = bx / nbx, i = blockIdx.y;
  const uint32_t gb = bx - tq * nbx;                    // this workgroup's 64 groups
  const uint32_t k = gb * kCol3Threads + threadIdx.x;   // float4 column of the stitched row
  const uint32_t cols = 3 * (uint32_t)a.nco, bank = k / cols, c = k - bank * cols;
  const bool in = bank < (uint32_t)a.nbank;
  const float id = R<OP>::id();
  const float4 id4 = make_float4(id, id, id, id);
  const int64_t ld = a.in_ld_t, tp0 = (int64_t)tq * TPB;
  const int nbp = (int)min((int64_t)TPB, a.nto - tp0);
  const float *p = a.in[in ? bank : 0] + a.in_off + (int64_t)i * a.in_ld_i + tp0 * T * ld + 4 * c;
  float4 v[NR];
  if (in && nbp == TPB) {
#pragma unroll
    for (int u = 0; u < NR; ++u) v[u] = ld4(p + u * ld);
  } else {
#pragma unroll
    for (int u = 0; u < NR; ++u) v[u] = (in && u < nbp * T) ? ld4(p + u * ld) : id4;
  }
  __shared__ float part[TPB][kCol3Threads];
#pragma unroll
  for (int b = 0; b < TPB; ++b) {
    float4 acc = id4;
#pragma unroll
    for (int r = 0; r < T; ++r) acc = f4<OP>(acc, v[b * T + r]);
    part[b][threadIdx.x] = fold4<OP>(acc);
  }
  __syncthreads();
  const int64_t ng = (int64_t)a.nbank * a.nco;  // groups of the stitched row
  for (int e = threadIdx.x; e < TPB * 64; e += kCol3Threads) {
    const int b = e >> 6, q = e & 63;
    const int64_t G = (int64_t)gb * 64 + q;
    if (b >= nbp || G >= ng) continue;
    const float s = R<OP>::f(R<OP>::f(part[b][3 * q], part[b][3 * q + 1]), part[b][3 * q + 2]);
    const int64_t bk = G / a.nco, g = G - bk * a.nco;
    st1<1>(a.out + bk * a.out_bank + (int64_t)i * a.out_ld_i + (tp0 + b) * a.out_ld_t + g,
           finish<OP>(s, a));
  }
}

// ---------------------------------------------------------------------------
// Scalar path: any F, any channel step, any alignment.  One lane per output.
template <int OP>
__device__ __forceinline__ void scalar_tile(const RedArgs &a, int64_t tile) {
  const Coord c = decompose(a, tile);
  const int64_t co = c.bc * kBlock + threadIdx.x;
  if (co >= a.nco) return;
  const int64_t r0 = c.chunk * a.rows_per_chunk;
  const int64_t r1 = min(a.T, r0 + a.rows_per_chunk);
  float acc[4] = {R<OP>::id(), R<OP>::id(), R<OP>::id(), R<OP>::id()};
  const float *p = a.in[c.bank] + a.in_off + c.i * a.in_ld_i + (c.to * a.T + r0) * a.in_ld_t +
                   co * a.F * a.in_cs;
  const int64_t cs = a.in_cs;
  for (int64_t r = r0; r < r1; ++r) {
    int64_t k = 0;
    for (; k + 4 <= a.F; k += 4) {
      float v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = p[(k + u) * cs];
#pragma unroll
      for (int u = 0; u < 4; ++u) acc[u] = R<OP>::f(acc[u], v[u]);
    }
    for (; k < a.F; ++k) acc[0] = R<OP>::f(acc[0], p[k * cs]);
    p += a.in_ld_t;
  }
  const float s = R<OP>::f(R<OP>::f(acc[0], acc[1]), R<OP>::f(acc[2], acc[3]));
  if (a.nchunk == 1)
    st1(a.out + c.bank * a.out_bank + c.i * a.out_ld_i + c.to * a.out_ld_t + co, finish<OP>(s, a));
  else
    a.ws[(((c.chunk * a.nbank + c.bank) * a.nto + c.to) * a.ni + c.i) * a.nco + co] = s;
}

// ---------------------------------------------------------------------------
// Tile path: channel step cs in 1..8, any F that fits a tile, any channel
// alignment (e.g. idxs = (1000:2023, :, :)), aligned row pitches.  Time
// integration is element-wise, so a workgroup streams the 16-byte-aligned
// superset of its tile's channels (gpt groups = gpt*F window channels, at most
// kSpan floats of a row) with 1 KiB-per-wave float4 loads, sums the T rows of
// every channel in registers, then drops the selected channels into LDS and
// folds each group of F there: 16-channel segments first, then the segments
// of a group.  HBM traffic is the window plus <= 3 floats per tile row edge.
// (A/B of 2 columns per thread and of one accumulator set: +-4%,
// profiles/r01_ab_tile.json)
constexpr int kTK = 4;                   // float4 columns per thread (a tile row: 1024 * kTK floats)
constexpr int kTA = 2;                   // accumulator sets per column
constexpr int kTRB = kBatch / kTK > 0 ? kBatch / kTK : 1;  // rows per load batch
constexpr int kSpan = kBlock * 4 * kTK;  // floats of one row one tile may read
constexpr int kSeg = 16;                 // channels folded per thread in stage 1
__device__ __forceinline__ int lpad(int x) { return x + (x >> 4); }  // LDS bank spread

template <int OP, bool CS1>
__device__ __forceinline__ void tile_tile(const RedArgs &a, int64_t tile) {
  __shared__ float lds[kSpan + kSpan / 16];
  __shared__ float part[2 * kBlock];
  const Coord c = decompose(a, tile);
  const int tid = threadIdx.x;
  const int64_t co0 = c.bc * a.gpt;  // first output channel of the tile
  const int gt = (int)min<int64_t>(a.gpt, a.nco - co0);
  const int F = (int)a.F;
  const int cs = CS1 ? 1 : (int)a.in_cs;
  const int ncht = gt * F;  // window channels of the tile
  const int64_t abs0 = a.in_off + c.i * a.in_ld_i + co0 * a.F * cs;
  const int mis = (int)(abs0 & 3);  // row pitches are multiples of 4 floats
  const int w4 = (mis + (ncht - 1) * cs + 1 + 3) >> 2;
  const int64_t r0 = c.chunk * a.rows_per_chunk;
  const int64_t r1 = min(a.T, r0 + a.rows_per_chunk);
  const float id = R<OP>::id();
  const float4 id4 = make_float4(id, id, id, id);
  const float *p = a.in[c.bank] + (abs0 - mis) + (c.to * a.T + r0) * a.in_ld_t + 4 * tid;
  const int64_t st = a.in_ld_t;

  float4 acc[kTA][kTK];
#pragma unroll
  for (int q = 0; q < kTA; ++q)
#pragma unroll
    for (int k = 0; k < kTK; ++k) acc[q][k] = id4;
  int64_t nrows = r1 - r0;
  for (; nrows >= kTRB; nrows -= kTRB) {
    float4 v[kTRB][kTK];
#pragma unroll
    for (int u = 0; u < kTRB; ++u)
#pragma unroll
      for (int k = 0; k < kTK; ++k)
        v[u][k] = (tid + k * kBlock < w4) ? ld4(p + u * st + 4 * k * kBlock) : id4;
    p += kTRB * st;
#pragma unroll
    for (int u = 0; u < kTRB; ++u)
#pragma unroll
      for (int k = 0; k < kTK; ++k) acc[u % kTA][k] = f4<OP>(acc[u % kTA][k], v[u][k]);
  }
  for (; nrows > 0; --nrows) {
#pragma unroll
    for (int k = 0; k < kTK; ++k)
      if (tid + k * kBlock < w4) acc[0][k] = f4<OP>(acc[0][k], ld4(p + 4 * k * kBlock));
    p += st;
  }
#pragma unroll
  for (int q = 1; q < kTA; ++q)
#pragma unroll
    for (int k = 0; k < kTK; ++k) acc[0][k] = f4<OP>(acc[0][k], acc[q][k]);
#pragma unroll
  for (int k = 0; k < kTK; ++k) {
    const int col = tid + k * kBlock;
    if (col >= w4) continue;
    const float4 r = acc[0][k];
    const float e[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int x = 4 * col + q - mis;  // element offset from the tile's first channel
      if (x < 0) continue;
      int ch = x;
      if (!CS1) {
        if (x % cs) continue;
        ch = x / cs;
      }
      if (ch < ncht) lds[lpad(ch)] = e[q];
    }
  }
  __syncthreads();

  auto store = [&](int g, float s) {
    const int64_t co = co0 + g;
    if (a.nchunk == 1)
      st1(a.out + c.bank * a.out_bank + c.i * a.out_ld_i + c.to * a.out_ld_t + co, finish<OP>(s, a));
    else
      a.ws[(((c.chunk * a.nbank + c.bank) * a.nto + c.to) * a.ni + c.i) * a.nco + co] = s;
  };
  if (F <= kSeg) {
    for (int g = tid; g < gt; g += kBlock) {
      float s = id;
      for (int k = 0; k < F; ++k) s = R<OP>::f(s, lds[lpad(g * F + k)]);
      store(g, s);
    }
  } else {
    const int nseg = (F + kSeg - 1) / kSeg;  // gt * nseg <= 2 * kBlock (F > kSeg)
    for (int q = tid; q < gt * nseg; q += kBlock) {
      const int g = q / nseg, sg = q - g * nseg;
      const int x0 = g * F + sg * kSeg, x1 = min(x0 + kSeg, g * F + F);
      float s = id;
      for (int x = x0; x < x1; ++x) s = R<OP>::f(s, lds[lpad(x)]);
      part[q] = s;
    }
    __syncthreads();
    for (int g = tid; g < gt; g += kBlock) {
      float s = id;
      for (int sg = 0; sg < nseg; ++sg) s = R<OP>::f(s, part[g * nseg + sg]);
      store(g, s);
    }
  }
  __syncthreads();  // lds/part are reused by the next tile of a grid-stride loop
}

// Grid-stride wrappers: one tile per workgroup when the grid covers every
// tile, several when a launch has more tiles than INT32_MAX workgroups; the
// first tile of a workgroup in the per-XCD order where the plan chose it.
template <int OP, int LPG, int K4C>
__global__ __launch_bounds__(kBlock) void k_reduce_vec(const RedArgs a) {
  const int64_t t0 = xcd_order(blockIdx.x, gridDim.x, a.xcd_lg);
  for (int64_t t = t0; t < a.ntiles; t += gridDim.x) vec_tile<OP, LPG, K4C>(a, t);
}

// Vector path, interleaved (PATH_VEC_IL): groups of F = 256*K4 channels
// (K4 = 2, 4, 8, 16 float4 per lane per row; F = 512 .. 4096, the 0000
// product's fqavby = 1024 among them), one time block per tile.  A workgroup
// owns GPW consecutive groups; its 4 waves interleave their loads so that every
// workgroup-instruction reads 4 KiB contiguous (thread tid reads float4
// 256*j + tid of the segment) instead of each wave streaming its own group
// (hbm_ceiling: 7.15 vs 7.09 TB/s on the cfg3 row pattern).  Slot j of a lane
// belongs to group (4*j + wave)/K4; every group is folded over lanes
// (xor butterfly), then over waves through LDS in wave order (deterministic).
// Grid: x = GPW-group segment, y = (IF, time block), z = bank: no 64-bit
// division on the way to the first load.
// Plan option "vec_il": 1 (default) = use it where it applies; 0 = k_reduce_vec.
//   kIlGpw       groups per workgroup: 2 (+0.4% on the 0000 band, +1.3% on one
//                bank, i.e. one rank at N=8, against 4)
//   kIlInflight  16-byte loads a lane issues per batch (power of two); 4
//                measured +0.1..0.7% against 8 on 1-, 2- and 8-bank launches
constexpr int kIlGpw = 2, kIlInflight = 4, kIlGpwK2 = 4;
// groups per workgroup for K4 float4 per lane per row: kIlGpwK2 = 4 at K4 = 2
// (fqavby = 512: two loads per lane per row, as fqavby = 1024 has with 2),
// +7% on the 0000 band and +6% on the 0002 band at fqavby 512, F = 1024
// unchanged (round 5, capped at 2 workgroups per CU, profiles/r05/
// ab_il_r05g.json)
constexpr int il_gpw(int k4) { return k4 == 2 ? kIlGpwK2 : kIlGpw; }
//   kIlShm       dynamic LDS bytes per workgroup, an allocation that caps the
//                workgroups resident per CU at 2 (160 KiB of LDS per CU):
//                32 KiB of loads in flight per CU instead of ~128 KiB (8
//                workgroups).  cfg3 4.886 -> 4.629 ms (+5.3%), one bank
//                +5.5%, tavby 8 +7.1%, the 0002 band at fqavby 1024 +3%; 3 per
//                CU +1%, 4 per CU +0%, 8 loads in flight per lane at 2 per CU
//                +1% (profiles/r05/ab_il_r05b.json).  Uncapped, SQ counters
//                showed 27.5 waves per CU with 53% of their cycles stalled on
//                issue (VMEM queues full), where the pure read's best form
//                runs 4 waves per CU 81% parked on s_waitcnt
//                (profiles/r05/cfg3_sq_summary_r05a.json).
constexpr unsigned kIlShm = 65536;
// One tile (GPW groups x one (IF, time block) x one bank) of the interleaved
// path.
template <int OP, int K4, int GPW, int IF>
__device__ __forceinline__ void il_tile(const RedArgs &a, int64_t bx, uint32_t it, int bank) {
  constexpr int NI = GPW * K4 / 4;           // loads per lane per row
  constexpr int PER = K4 < 4 ? 1 : K4 / 4;   // consecutive loads of one group slot
  constexpr int NS = NI / PER;               // group slots per lane
  constexpr int RB = NI < IF ? IF / NI : 1;  // rows in flight
  constexpr int JB = NI < IF ? NI : IF;      // loads per batch within a row
  static_assert(NI >= 1 && NI % PER == 0, "k_reduce_il: GPW * K4 must be a multiple of 4");
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const uint32_t ni = (uint32_t)a.ni;
  const uint32_t to = it / ni, i = it - to * ni;
  const int64_t g0 = bx * GPW;
  const int ng = (int)min((int64_t)GPW, a.nco - g0);
  const float id = R<OP>::id();
  float4 acc[NS];
#pragma unroll
  for (int q = 0; q < NS; ++q) acc[q] = make_float4(id, id, id, id);
  const float *p = a.in[bank] + a.in_off + (int64_t)i * a.in_ld_i +
                   (int64_t)to * a.T * a.in_ld_t + g0 * a.F + 4 * tid;
  const int64_t ld = a.in_ld_t;
  auto slot = [&](int j) { return j / PER; };
  auto group = [&](int j) { return (4 * j + wave) / K4; };
  int64_t nrows = a.T;
  if (ng == GPW) {
    if constexpr (NI < 8) {
      for (; nrows >= RB; nrows -= RB) {
        float4 v[RB * NI];
#pragma unroll
        for (int u = 0; u < RB; ++u)
#pragma unroll
          for (int j = 0; j < NI; ++j) v[u * NI + j] = ld4(p + u * ld + 1024 * j);
        p += RB * ld;
#pragma unroll
        for (int u = 0; u < RB; ++u)
#pragma unroll
          for (int j = 0; j < NI; ++j) acc[slot(j)] = f4<OP>(acc[slot(j)], v[u * NI + j]);
      }
    }
    for (; nrows > 0; --nrows) {
#pragma unroll
      for (int jb = 0; jb < NI; jb += JB) {
        float4 v[JB];
#pragma unroll
        for (int j = 0; j < JB; ++j) v[j] = ld4(p + 1024 * (jb + j));
#pragma unroll
        for (int j = 0; j < JB; ++j) acc[slot(jb + j)] = f4<OP>(acc[slot(jb + j)], v[j]);
      }
      p += ld;
    }
  } else {  // last segment of a row with fewer than GPW groups: skip absent ones
    for (; nrows > 0; --nrows) {
#pragma unroll
      for (int j = 0; j < NI; ++j)
        if (group(j) < ng) acc[slot(j)] = f4<OP>(acc[slot(j)], ld4(p + 1024 * j));
      p += ld;
    }
  }
  __shared__ float red[4][NS];
#pragma unroll
  for (int q = 0; q < NS; ++q) {
    const float s = lanes_fold<OP, 64>(fold4<OP>(acc[q]));
    if (lane == 0) red[wave][q] = s;
  }
  __syncthreads();
  if (tid < ng) {
    float s = id;
#pragma unroll
    for (int w = 0; w < 4; ++w)
#pragma unroll
      for (int q = 0; q < NS; ++q)
        if ((4 * q * PER + w) / K4 == tid) s = R<OP>::f(s, red[w][q]);
    st1o(a.out + bank * a.out_bank + (int64_t)i * a.out_ld_i + (int64_t)to * a.out_ld_t + g0 + tid,
         finish<OP>(s, a), a.st_plain);
  }
}

template <int OP, int K4, int GPW>
__global__ __launch_bounds__(kBlock) void k_reduce_il(const RedArgs a) {
  il_tile<OP, K4, GPW, kIlInflight>(a, xcd_order(blockIdx.x, gridDim.x, a.xcd_lg), blockIdx.y,
                                    blockIdx.z);
}

// Vector path, small groups (PATH_VEC_ROW): F = 4*G4 channels with G4 = 1..64
// float4 (F = 4 .. 256, e.g. the 0002 product's fqavby = 64), one float4
// column per lane, one time block per tile.  A workgroup owns 1024
// consecutive window channels (256 / G4 groups) of one (IF, time block,
// bank); a workgroup-instruction reads 4 KiB contiguous, 8 rows are in flight
// per lane, and each group folds over its G4 lanes with an xor butterfly
// (groups never straddle a wave).  The lean sibling of k_reduce_vec for
// these plans: 3-D grid, no 64-bit division, no time split.
// Plan option "vec_row": 1 (default) = use it where it applies; 0 =
// k_reduce_vec.  kRowBatch rows in flight per lane: 16 (+2.6% / +3.2% on the
// 0002 band / bank against 8, -0.4% on 0000 F=64, -1.7% on 0001 F=64).  At
// most kRowMaxWaves = 4 resident waves per SIMD: fewer 4 KiB row streams per
// CU in flight is faster on the 0002 shapes (A/B against uncapped /
// k_reduce_vec: cfg1 5.85 vs 5.59 / 5.43 TB/s, cfg2 6.18 vs 5.78 / 6.10).
constexpr int kRowBatch = 16;
template <int OP, int G4>
__global__ __launch_bounds__(kBlock)
__attribute__((amdgpu_waves_per_eu(1, kRowMaxWaves)))
void k_reduce_row(const RedArgs a) {
  const int tid = threadIdx.x;
  const uint32_t it = blockIdx.y, ni = (uint32_t)a.ni;
  const uint32_t to = it / ni, i = it - to * ni;
  const int bank = blockIdx.z;
  const int64_t col = (int64_t)xcd_order(blockIdx.x, gridDim.x, a.xcd_lg) * kBlock + tid;  // float4 column of the window
  const bool valid = col < a.nco * G4;
  const float id = R<OP>::id();
  float4 acc[kNacc];
#pragma unroll
  for (int q = 0; q < kNacc; ++q) acc[q] = make_float4(id, id, id, id);
  if (valid) {
    const float *p = a.in[bank] + a.in_off + (int64_t)i * a.in_ld_i +
                     (int64_t)to * a.T * a.in_ld_t + 4 * col;
    const int64_t ld = a.in_ld_t;
    int64_t nrows = a.T;
    for (; nrows >= kRowBatch; nrows -= kRowBatch) {
      float4 v[kRowBatch];
#pragma unroll
      for (int u = 0; u < kRowBatch; ++u) v[u] = ld4(p + u * ld);
      p += kRowBatch * ld;
#pragma unroll
      for (int u = 0; u < kRowBatch; ++u) acc[u % kNacc] = f4<OP>(acc[u % kNacc], v[u]);
    }
    acc[0] = tail_rows<OP, kRowBatch>(acc[0], p, ld, nrows);
  }
  const float s = lanes_fold<OP, G4>(fold4<OP>(fold_acc<OP>(acc)));
  if (valid && (tid & (G4 - 1)) == 0)
    st1o(a.out + bank * a.out_bank + (int64_t)i * a.out_ld_i + (int64_t)to * a.out_ld_t + col / G4,
         finish<OP>(s, a), a.st_plain);
}

// k_reduce_row with a time block's rows split over S slices of the
// workgroup (S = 2, 4; T a multiple of 16): 256 / S float4 columns per
// workgroup, S times the workgroups.  A launch of one file (one 0002 bank at
// fqavby = 64, tavby = 16: 1088 row tiles of 64 KiB on 256 CUs) otherwise
// ends on a partial round of workgroups.  Slice s keeps k_reduce_row's
// accumulators s*8/S .. (s+1)*8/S - 1, i.e. exactly the rows k_reduce_row adds
// into them (row r of every 16-row batch goes to accumulator r % 8), in the
// same order; slice 0 collects the others' accumulators through LDS and runs
// k_reduce_row's folds, so the results are bit-identical to it.
template <int OP, int G4, int S>
__global__ __launch_bounds__(kBlock)
__attribute__((amdgpu_waves_per_eu(1, kRowMaxWaves)))
void k_reduce_rows(const RedArgs a) {
  constexpr int CW = kBlock / S;      // float4 columns per workgroup
  constexpr int NA = kNacc / S;       // accumulators per slice
  constexpr int RPB = 16 / S;         // rows per 16-row batch per slice
  static_assert(kNacc == 8 && kRowBatch == 16, "k_reduce_rows mirrors k_reduce_row's 16 x 8");
  static_assert(CW >= 64 && G4 <= 64, "groups never straddle a wave");
  const int tid = threadIdx.x;
  const int sl = tid / CW, c = tid - sl * CW;  // slice (wave-uniform), column within the workgroup
  const uint32_t it = blockIdx.y, ni = (uint32_t)a.ni;
  const uint32_t to = it / ni, i = it - to * ni;
  const int bank = blockIdx.z;
  const int64_t col = (int64_t)xcd_order(blockIdx.x, gridDim.x, a.xcd_lg) * CW + c;  // float4 column of the window
  const bool valid = col < a.nco * G4;
  const float id = R<OP>::id();
  float4 acc[NA];
#pragma unroll
  for (int q = 0; q < NA; ++q) acc[q] = make_float4(id, id, id, id);
  if (valid) {
    // slice sl owns accumulators sl*NA .. sl*NA + NA - 1: rows
    // 8h + sl*NA + q (h = 0, 1) of every 16-row batch
    const float *p = a.in[bank] + a.in_off + (int64_t)i * a.in_ld_i +
                     ((int64_t)to * a.T + sl * NA) * a.in_ld_t + 4 * col;
    const int64_t ld = a.in_ld_t;
    for (int64_t nb = a.T / 16; nb > 0; --nb) {
      float4 v[RPB];
#pragma unroll
      for (int u = 0; u < RPB; ++u) v[u] = ld4(p + ((u / NA) * 8 + u % NA) * ld);
      p += 16 * ld;
#pragma unroll
      for (int u = 0; u < RPB; ++u) acc[u % NA] = f4<OP>(acc[u % NA], v[u]);
    }
  }
  __shared__ float4 xs[S - 1][NA][CW];
  if (sl > 0) {
#pragma unroll
    for (int q = 0; q < NA; ++q) xs[sl - 1][q][c] = acc[q];
  }
  __syncthreads();
  if (sl == 0) {
    float4 all[kNacc];
#pragma unroll
    for (int q = 0; q < NA; ++q) all[q] = acc[q];
#pragma unroll
    for (int s2 = 1; s2 < S; ++s2)
#pragma unroll
      for (int q = 0; q < NA; ++q) all[s2 * NA + q] = xs[s2 - 1][q][c];
    const float s = lanes_fold<OP, G4>(fold4<OP>(fold_acc<OP>(all)));
    if (valid && (c & (G4 - 1)) == 0)
      st1o(a.out + bank * a.out_bank + (int64_t)i * a.out_ld_i + (int64_t)to * a.out_ld_t +
               col / G4,
           finish<OP>(s, a), a.st_plain);
  }
}

// The row path for short time blocks (T = 1, 2, 4: tavby = 1 is the
// reference's own fqav, src/gbtworkerfunctions.jl:16-20, with no time
// integration).  k_reduce_row gives every workgroup one time block, so at T = 1
// a workgroup reads a single 4 KiB row segment and the launch is dominated by
// workgroup turnover (3.1 TB/s on the 0002 band at F = 16).  Here a workgroup
// takes TPB = 16 / T consecutive time blocks of its 1024 channels: 16 rows in
// flight per lane, as k_reduce_row at T = 16.  Each block is summed exactly as
// k_reduce_row sums it (rows chained into the first accumulator, the same
// folds), so the results are bit-identical to it.
// Plan options: "row_tpb" 1 (default) = use it for T in {1, 2, 3, 4, 8}; 0 =
// k_reduce_row.  "rowt_pack" 1 (default) = windows of <= 128 float4 columns
// share a workgroup between 2 or 4 time groups (no idle lanes).  "rowt_small"
// (64): launches that would have fewer than this many workgroups per CU with
// 16 rows per lane take 8 rows per lane (TPB = 8 / T, twice the workgroups),
// 4 at T <= 2 (round 4; 0 = always 16).  A/B, profiles/r03/ab_rowt_r03i.json
// (bit-identical): 8 rows win on one 0002 file (1152 workgroups, 4.5 per CU:
// +10-18% at F = 16..256, T = 1, 2, 4) and on the 0002 band (9216: +1.5-3.5%),
// and lose on the 0000 band (>= 200k workgroups: -1.5-3.5%); 4 rows another
// 2-6% on the 0002 band at T = 1, 2 (profiles/r04/ab_grid_r04x.json).
// "rowt_narrow8": the 0001 product's <= 128-column windows take 8 rows too at
// T = 1 and F >= 64; "row_bpack": on a stitched band of such windows the two
// lane sets take two banks (template form BP).  The output tile is staged
// in LDS and stored as whole row segments (16-byte stores where legal; each
// wave storing its own groups' outputs was slower).  At most kRowtMaxWaves = 6
// resident waves per SIMD (A/B against 4 and none, profiles/r02/ab_row_tpb.json).
template <int OP, int G4, int T, int NRW, bool BP>
__global__ __launch_bounds__(kBlock)
__attribute__((amdgpu_waves_per_eu(1, kRowtMaxWaves)))
void k_reduce_rowt(const RedArgs a) {
  constexpr int TPB = NRW / T, NR = TPB * T;
  const int tid = threadIdx.x;
  // grid: x = (column block, time group) column block fastest, y = IF, z = bank.
  // Windows of <= 128 float4 columns (the 512-channel 0001 product) share a
  // workgroup between 2^tsub_log2 time groups, 256 >> tsub_log2 lanes each.
  // With a.bpack the 2^tsub_log2 lane sets take 2^tsub_log2 consecutive banks
  // of one time group instead (grid z = bank sets): a stitched product's rows
  // then get whole segments of 2^tsub_log2 banks' outputs (below).
  const uint32_t bx = xcd_order(blockIdx.x, gridDim.x, a.xcd_lg);
  const uint32_t bc = (uint32_t)a.blocks_c;
  const int sh = a.tsub_log2, cw = kBlock >> sh, sub = threadIdx.x >> (8 - sh);  // (kBlock = 256)
  constexpr bool bp = BP;  // (a.bpack: a template form, so the time-group form pays nothing)
  const uint32_t tq = bx / bc, i = blockIdx.y;
  const int64_t tg = bp ? (int64_t)tq : ((int64_t)tq << sh) + sub;
  const int bank = bp ? (int)(blockIdx.z << sh) + sub : (int)blockIdx.z;
  const int64_t col = (int64_t)(bx - tq * bc) * kBlock + (tid & (cw - 1));  // float4 column
  const int64_t to0 = tg * TPB;
  const bool valid = col < a.nco * G4 && to0 < a.nto;
  // time blocks of this lane's group (uniform over each wave: groups hold >= 64 lanes)
  const int nb = (int)max((int64_t)0, min((int64_t)TPB, a.nto - to0));
  const float id = R<OP>::id();
  const float4 id4 = make_float4(id, id, id, id);
  const float *p = a.in[bank] + a.in_off + (int64_t)i * a.in_ld_i + to0 * T * a.in_ld_t + 4 * col;
  const int64_t ld = a.in_ld_t;
  float4 v[NR];
  if (valid && nb == TPB) {  // every tile but the last time group: no predication
#pragma unroll
    for (int u = 0; u < NR; ++u) v[u] = ld4(p + u * ld);
  } else {
#pragma unroll
    for (int u = 0; u < NR; ++u) v[u] = (valid && u < nb * T) ? ld4(p + u * ld) : id4;
  }
  // k_reduce_row's accumulators for a block of T < 16 rows: the rows chained
  // into the first, the others left at the identity; its pairwise fold of
  // them then amounts to one more op with the identity (f is idempotent
  // there), which is all that is done here.  Every lane of a group ends with
  // the group's sums of all TPB blocks (lanes_fold).
  float sv[TPB];
#pragma unroll
  for (int b = 0; b < TPB; ++b) {
    float4 acc = id4;
#pragma unroll
    for (int r = 0; r < T; ++r) acc = f4<OP>(acc, v[b * T + r]);
    if constexpr (kNacc > 1) acc = f4<OP>(acc, id4);
    sv[b] = lanes_fold<OP, G4>(fold4<OP>(acc));
  }
  // Output tile through LDS: the workgroup's outputs are (time groups x TPB)
  // rows of 256/G4 >> tsub_log2 consecutive groups.  Lane j of a group
  // deposits block j (j + G4, ...); then each row segment is stored by
  // consecutive lanes, 16 bytes per lane where the output layout allows, so
  // every row segment leaves the CU as whole writes (storing per wave put 4
  // pieces of each 64-byte segment in flight at F = 64, and 1 float per
  // wave per row at F = 256: 32-byte partial write requests, PMC WRITE_SIZE
  // 2x-5x the output, profiles/r03/t1_pmc_r03a.json).
  __shared__ float tile[kBlock / G4 * TPB];
  const int j = tid & (G4 - 1);
  constexpr int NS = TPB > G4 ? (TPB + G4 - 1) / G4 : 1;  // (TPB = 5 at T = 3)
  constexpr int NSEL = TPB < G4 ? TPB : G4;
  constexpr int LG4 = G4 >= 64 ? 6 : G4 >= 32 ? 5 : G4 >= 16 ? 4 : G4 >= 8 ? 3 : G4 >= 4 ? 2 : G4 >= 2 ? 1 : 0;
  const int lng = 8 - sh - LG4;  // log2 of the groups per row segment (>= 0: cw >= G4)
  const int gl = (tid & (cw - 1)) >> LG4;
#pragma unroll
  for (int m = 0; m < NS; ++m) {
    const int b = m * G4 + j;
    float val = sv[m * G4];
#pragma unroll
    for (int q = 1; q < NSEL; ++q)
      if (m * G4 + q < TPB) val = (j == q) ? sv[m * G4 + q] : val;
    // tile rows: (time group, block) pairs, or with bpack one row per block
    // holding the bank sets' segments side by side (nco = 2^lng: contiguous
    // in the stitched product, whose banks are nco outputs apart)
    if (b < TPB) tile[((bp ? (b << sh) + sub : sub * TPB + b) << lng) + gl] = finish<OP>(val, a);
  }
  __syncthreads();
  const int64_t gcol0 = (int64_t)(bx - tq * bc) * (kBlock / G4);
  float *ob = a.out + (int64_t)(bp ? (int)(blockIdx.z << sh) : bank) * a.out_bank +
              (int64_t)i * a.out_ld_i + gcol0;
  const int nrow = bp ? TPB : TPB << sh;
  const int lw = bp ? lng + sh : lng;  // log2 of a tile row's outputs
  const int64_t lim = bp ? a.nco << sh : a.nco, tob = bp ? (int64_t)tq * TPB : ((int64_t)tq << sh) * TPB;
  if (a.vec_out && lw >= 2) {
    const int lq = lw - 2;  // log2 of the float4 per row segment
    for (int e = tid; e < (nrow << lq); e += kBlock) {
      const int r = e >> lq, q = e & ((1 << lq) - 1);
      const int64_t to = tob + r;  // r = sub * TPB + b (bpack: r = b)
      const int64_t g = gcol0 + 4 * q;
      if (to >= a.nto || g >= lim) continue;
      const float *src = &tile[(r << lw) + 4 * q];
      float *dst = ob + to * a.out_ld_t + 4 * q;
      if (g + 3 < lim) {
        st4o(dst, make_float4(src[0], src[1], src[2], src[3]), a.st_plain);
      } else {
        for (int k = 0; k < 4; ++k)
          if (g + k < lim) st1o(dst + k, src[k], a.st_plain);
      }
    }
  } else {
    for (int e = tid; e < (nrow << lw); e += kBlock) {
      const int r = e >> lw, q = e & ((1 << lw) - 1);
      const int64_t to = tob + r;
      if (to >= a.nto || gcol0 + q >= lim) continue;
      st1o(ob + to * a.out_ld_t + q, tile[e], a.st_plain);
    }
  }
  (void)valid;
}

// Large groups (F = 512..4096: 64 lanes x K4 float4 per row, one output per
// wave per time block) with short time blocks (T = 1, 2, 4) on windows where
// the interleaved kernel is a poor fit (few groups per row, or more (IF, time
// block) pairs than its 3-D grid holds): e.g. fqavby = 512 on the 512-channel
// 0001 product, one output per spectrum, which k_reduce_vec ran one row per
// 4-wave workgroup (0.95 TB/s).  Each wave owns one group and RW consecutive
// time blocks, TB of them per batch (>= 16 loads per lane in flight); a time
// block is summed exactly as k_reduce_vec sums it (its batched and remainder
// accumulator patterns, the same folds), so the results are bit-identical.
// Plan option "wavet": 1 (default) = use it where the interleaved kernel
// cannot run or a row holds fewer than 4 groups; 2 = for every such shape;
// 0 = never.
// BP (plan option "wave_bpack"): a stitched band whose product row is <= 16
// groups (the 0001 band at fqavby = 512: one output per bank per spectrum) is
// reduced by workgroups of one wave per (bank, group) of the row, all on the
// same time blocks; their outputs go through LDS and leave as whole product
// rows, contiguous over the workgroup's RW spectra, where each wave storing
// its own put 4 bytes into every 32-byte row.
template <int OP, int K4, int T, bool BP>
__global__ __launch_bounds__(BP ? 1024 : kBlock) void k_reduce_wavet(const RedArgs a) {
  constexpr int TB = (16 / (T * K4)) > 0 ? 16 / (T * K4) : 1;  // time blocks per batch
  // batches per wave: one where a batch holds >= 2 time blocks (the 0001
  // band at fqavby = 512: 2.75 -> 2.31 ms at T = 1, +3..19% at T = 2..4 and
  // on long windows at F = 1024, 2048; profiles/r04/ab_wavet_r04g.json), else
  // 4 (one block per batch: 4 batches measured faster than 2 at F = 4096)
  constexpr int NBAT = TB >= 2 ? 1 : 4, RW = TB * NBAT;
  // k_reduce_vec's accumulation of one time block: K4 in {2, 4} take RB-row
  // batches (accumulator (u * K4 + k) % kNacc) then single rows (k % kNacc);
  // K4 >= 8 always the latter
  constexpr int RB = (K4 == 2 || K4 == 4) ? (K4 >= kBatch ? 1 : kBatch / K4) : 0;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t bx = xcd_order(blockIdx.x, gridDim.x, a.xcd_lg);
  const int64_t g = BP ? wave % a.nco : bx % a.nco, chunk = BP ? bx : bx / a.nco;
  const int64_t i = blockIdx.y;
  const int bank = BP ? (int)(wave / a.nco) : (int)blockIdx.z;
  const int64_t tb0 = BP ? chunk * RW : (chunk * 4 + wave) * RW;
  __shared__ float tile[BP ? RW * 16 : 1];  // (BP: RW rows of <= 16 outputs)
  const int W = BP ? (int)(blockDim.x >> 6) : 0;
  const float id = R<OP>::id();
  const float *base = a.in[bank] + a.in_off + i * a.in_ld_i + g * a.F + 4 * lane;
  const int64_t ld = a.in_ld_t;
  for (int bt = 0; bt < NBAT; ++bt) {
    const int64_t t0 = tb0 + (int64_t)bt * TB;
    if (t0 >= a.nto) break;  // (uniform over the wave)
    const int nb = (int)min((int64_t)TB, a.nto - t0);
    float4 v[TB * T * K4];
#pragma unroll
    for (int b = 0; b < TB; ++b)
#pragma unroll
      for (int r = 0; r < T; ++r)
#pragma unroll
        for (int k = 0; k < K4; ++k)
          if (b < nb) v[(b * T + r) * K4 + k] = ld4(base + ((t0 + b) * T + r) * ld + 256 * k);
#pragma unroll
    for (int b = 0; b < TB; ++b) {
      if (b < nb) {
        float4 acc[kNacc];
#pragma unroll
        for (int q = 0; q < kNacc; ++q) acc[q] = make_float4(id, id, id, id);
        int r = 0;
        if constexpr (RB > 0) {
#pragma unroll
          for (; r + RB <= T; r += RB)
#pragma unroll
            for (int u = 0; u < RB; ++u)
#pragma unroll
              for (int k = 0; k < K4; ++k)
                acc[(u * K4 + k) % kNacc] =
                    f4<OP>(acc[(u * K4 + k) % kNacc], v[(b * T + r + u) * K4 + k]);
        }
#pragma unroll
        for (; r < T; ++r)
#pragma unroll
          for (int k = 0; k < K4; ++k)
            acc[k % kNacc] = f4<OP>(acc[k % kNacc], v[(b * T + r) * K4 + k]);
        const float s = lanes_fold<OP, 64>(fold4<OP>(fold_acc<OP>(acc)));
        if (lane == 0) {
          if constexpr (BP)
            tile[(bt * TB + b) * W + wave] = finish<OP>(s, a);
          else
            st1<1>(a.out + bank * a.out_bank + i * a.out_ld_i + (t0 + b) * a.out_ld_t + g,
                   finish<OP>(s, a));
        }
      }
    }
  }
  if constexpr (BP) {  // the RW product rows, W = nbank * nco outputs each (out_bank = nco)
    __syncthreads();
    const int64_t nr = min((int64_t)RW, a.nto - tb0);
    for (int e = threadIdx.x; e < nr * W; e += blockDim.x) {
      const int r = e / W, w = e - r * W;
      st1<1>(a.out + i * a.out_ld_i + (tb0 + r) * a.out_ld_t + w, tile[e]);
    }
  }
}

template <int OP, int F>
__global__ __launch_bounds__(kBlock) void k_reduce_narrow(const RedArgs a) {
  const int64_t t0 = xcd_order(blockIdx.x, gridDim.x, a.xcd_lg);
  for (int64_t t = t0; t < a.ntiles; t += gridDim.x) narrow_tile<OP, F>(a, t);
}
template <int OP, int F>
__global__ __launch_bounds__(kBlock) void k_reduce_narrow_mis(const RedArgs a) {
  for (int64_t t = blockIdx.x; t < a.ntiles; t += gridDim.x) narrow_mis_tile<OP, F>(a, t);
}
template <int OP, int F>
__global__ __launch_bounds__(kBlock) void k_reduce_lane(const RedArgs a) {
  for (int64_t t = blockIdx.x; t < a.ntiles; t += gridDim.x) lane_tile<OP, F>(a, t);
}
template <int OP>
__global__ __launch_bounds__(kBlock) void k_reduce_scalar(const RedArgs a) {
  for (int64_t t = blockIdx.x; t < a.ntiles; t += gridDim.x) scalar_tile<OP>(a, t);
}
// At most kTileMaxWaves = 3 resident waves per SIMD for k_reduce_tile (A/B
// against uncapped, 5 waves: +0.6 to +4.6% on the misaligned / odd-F windows;
// 2 is better on 0000-sized windows but 2.6% worse on a misaligned 0002 band).
template <int OP, bool CS1>
__global__ __launch_bounds__(kBlock)
__attribute__((amdgpu_waves_per_eu(1, kTileMaxWaves)))
void k_reduce_tile(const RedArgs a) {
  const int64_t t0 = xcd_order(blockIdx.x, gridDim.x, a.xcd_lg);
  for (int64_t t = t0; t < a.ntiles; t += gridDim.x) tile_tile<OP, CS1>(a, t);
}

// Second stage of a time-chunked reduction: fold the nchunk partials of every
// output in chunk order (deterministic), apply the mean divisor, scatter into
// the (possibly stitched) output layout.
template <int OP>
__device__ __forceinline__ void reduce_store(const RedArgs &a, int64_t e, float s) {
  int64_t r = e;
  const int64_t co = r % a.nco;
  r /= a.nco;
  const int64_t i = r % a.ni;
  r /= a.ni;
  const int64_t to = r % a.nto;
  const int64_t bank = r / a.nto;
  st1(a.out + bank * a.out_bank + i * a.out_ld_i + to * a.out_ld_t + co, finish<OP>(s, a));
}

template <int OP>
__global__ __launch_bounds__(kBlock) void k_reduce_finalize(const RedArgs a) {
  const int64_t per_chunk = (int64_t)a.nbank * a.nto * a.ni * a.nco;
  for (int64_t e = (int64_t)blockIdx.x * kBlock + threadIdx.x; e < per_chunk;
       e += (int64_t)gridDim.x * kBlock) {
    float s = a.ws[e];
    for (int ch = 1; ch < a.nchunk; ++ch) s = R<OP>::f(s, a.ws[ch * per_chunk + e]);
    reduce_store<OP>(a, e, s);
  }
}

// Many chunks, few outputs: one wave per output, lanes take chunks lane,
// lane+64, ... in order, then a fixed xor tree (deterministic).
template <int OP>
__global__ __launch_bounds__(kBlock) void k_reduce_finalize_w(const RedArgs a) {
  const int lane = threadIdx.x & 63;
  const int64_t per_chunk = (int64_t)a.nbank * a.nto * a.ni * a.nco;
  for (int64_t e = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); e < per_chunk;
       e += (int64_t)gridDim.x * 4) {
    float s = R<OP>::id();
    for (int ch = lane; ch < a.nchunk; ch += 64) s = R<OP>::f(s, a.ws[ch * per_chunk + e]);
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) s = R<OP>::f(s, __shfl_xor(s, off, 64));
    if (lane == 0) reduce_store<OP>(a, e, s);
  }
}

// ---------------------------------------------------------------------------
// Band stitch: bank-major gathered blocks -> vcat along channels.
__global__ __launch_bounds__(kBlock) void k_stitch4(int nbank, const float *__restrict__ g,
                                                    int64_t nc, int64_t nrows,
                                                    float *__restrict__ out) {
  const int64_t nc4 = nc / 4, wide4 = nc4 * nbank, n4 = wide4 * nrows;
  for (int64_t e = (int64_t)blockIdx.x * kBlock + threadIdx.x; e < n4;
       e += (int64_t)gridDim.x * kBlock) {
    const int64_t row = e / wide4, cw = e - row * wide4;
    const int64_t b = cw / nc4, c4 = cw - b * nc4;
    reinterpret_cast<float4 *>(out)[e] =
        reinterpret_cast<const float4 *>(g)[(b * nrows + row) * nc4 + c4];
  }
}
__global__ __launch_bounds__(kBlock) void k_stitch1(int nbank, const float *__restrict__ g,
                                                    int64_t nc, int64_t nrows,
                                                    float *__restrict__ out) {
  const int64_t wide = nc * nbank, n = wide * nrows;
  for (int64_t e = (int64_t)blockIdx.x * kBlock + threadIdx.x; e < n;
       e += (int64_t)gridDim.x * kBlock) {
    const int64_t row = e / wide, cw = e - row * wide;
    const int64_t b = cw / nc, c = cw - b * nc;
    out[e] = g[(b * nrows + row) * nc + c];
  }
}

// DC-spike patch: d[spike + k*nfpc] = d[spike - 1 + k*nfpc] per row.
__global__ __launch_bounds__(kBlock) void k_despike(float *d, int64_t nchan, int64_t nrows,
                                                    int64_t nfpc, int64_t nspike) {
  const int64_t n = nrows * nspike;
  const int64_t spike = nfpc / 2;
  for (int64_t e = (int64_t)blockIdx.x * kBlock + threadIdx.x; e < n;
       e += (int64_t)gridDim.x * kBlock) {
    const int64_t row = e / nspike, k = e - row * nspike;
    float *r = d + row * nchan + k * nfpc + spike;
    r[0] = r[-1];
  }
}

// ---------------------------------------------------------------------------
// Synthetic filterbank generator (counter-based, so any element is
// reproducible from (seed, index) alone).
__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}
__device__ __forceinline__ float synth_val(uint64_t e, int64_t nchan, int64_t nfpc,
                                           uint64_t seed, int kind) {
  const uint64_t h = splitmix64(e + seed * 0xD1B54A32D192ED03ull);
  if (kind == 1) return (float)(h >> 56);
  const float u1 = (float)((h >> 41) + 1) * (1.0f / 8388608.0f);
  const float u2 = (float)(((h >> 17) & 0x7FFFFF) + 1) * (1.0f / 8388608.0f);
  const float gam = -(logf(u1) + logf(u2)) * 5.0e8f;  // gamma(k=2, theta=5e8)
  const int64_t x = (int64_t)(e % (uint64_t)nchan) % nfpc;
  const float s = sinf(3.14159265f * ((float)x + 0.5f) / (float)nfpc);
  float bp = 0.2f + 0.8f * s * s;  // per-coarse-channel scallop
  if (x == nfpc / 2) bp *= 10.0f;  // DC spike (src/gbt.jl:102 position)
  return gam * bp;
}
__global__ __launch_bounds__(kBlock) void k_synth(float *out, int64_t n, int64_t nchan,
                                                  int64_t nfpc, uint64_t seed, int kind,
                                                  int vec) {
  const int64_t n4 = (n + 3) / 4;
  for (int64_t q = (int64_t)blockIdx.x * kBlock + threadIdx.x; q < n4;
       q += (int64_t)gridDim.x * kBlock) {
    const int64_t e = 4 * q;
    if (vec && e + 3 < n) {
      float4 v = make_float4(synth_val(e, nchan, nfpc, seed, kind),
                             synth_val(e + 1, nchan, nfpc, seed, kind),
                             synth_val(e + 2, nchan, nfpc, seed, kind),
                             synth_val(e + 3, nchan, nfpc, seed, kind));
      *reinterpret_cast<float4 *>(out + e) = v;
    } else {
      for (int64_t x = e; x < n && x < e + 4; ++x) out[x] = synth_val(x, nchan, nfpc, seed, kind);
    }
  }
}

int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }

// Timing events carried by the reduce's own dispatches (hipExtLaunchKernel,
// bldp_reduce_launch_timed): the start event takes the first dispatch's start
// and the stop event the last dispatch's end, with no marker packets queued
// between one launch and the next (a hipEventRecord pair costs a short launch
// a few microseconds of command-processor time).
thread_local hipEvent_t t_ev_start = nullptr, t_ev_stop = nullptr;

// SH: dynamic LDS bytes, here an occupancy cap (kIlShm, kRowShm, ...): a
// workgroup's allocation above 64 KiB needs the kernel's attribute raised.
#define BLDP_LAUNCH(KN, GR, BL, SH, ST, ...)                                          \
  do {                                                                                \
    if ((SH) > 65536u)                                                                \
      (void)hipFuncSetAttribute(reinterpret_cast<const void *>(KN),                   \
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)(SH)); \
    if (t_ev_stop) {                                                                  \
      hipExtLaunchKernelGGL(KN, GR, BL, SH, ST, t_ev_start, t_ev_stop, 0, __VA_ARGS__); \
      t_ev_start = nullptr;                                                           \
    } else {                                                                          \
      hipLaunchKernelGGL(KN, GR, BL, SH, ST, __VA_ARGS__);                            \
    }                                                                                 \
  } while (0)

template <int OP>
hipError_t launch_vec(const RedArgs &a, const Plan &p, hipStream_t s) {
  const dim3 grid((unsigned)p.grid), block(kBlock);
  const int k4c = (a.k4 == 1 || a.k4 == 2 || a.k4 == 4 || a.k4 == 3) ? a.k4 : 0;
#define BLDP_VEC(L, K)                                                 \
  if (p.lpg == L && k4c == K) {                                        \
    BLDP_LAUNCH((k_reduce_vec<OP, L, K>), grid, block, kVecShm, s, a); \
    return hipGetLastError();                                          \
  }
  BLDP_VEC(64, 1) BLDP_VEC(64, 2) BLDP_VEC(64, 4) BLDP_VEC(64, 0)
  BLDP_VEC(32, 1) BLDP_VEC(32, 0) BLDP_VEC(16, 1) BLDP_VEC(16, 0)
  BLDP_VEC(8, 1) BLDP_VEC(8, 0) BLDP_VEC(4, 1) BLDP_VEC(4, 0)
  BLDP_VEC(2, 1) BLDP_VEC(2, 0) BLDP_VEC(1, 1) BLDP_VEC(1, 0)
  BLDP_VEC(1, 3) BLDP_VEC(2, 3) BLDP_VEC(4, 3) BLDP_VEC(8, 3) BLDP_VEC(16, 3) BLDP_VEC(32, 3)
  BLDP_VEC(64, 3)
#undef BLDP_VEC
  return hipErrorInvalidValue;
}

template <int OP>
hipError_t launch_op(const RedArgs &a, const Plan &p, hipStream_t s) {
  hipError_t e = hipSuccess;
  const dim3 grid((unsigned)p.grid), block(kBlock);
  if (p.path == PATH_NARROW && a.tpb > 1) {  // short time blocks, several per workgroup
    const dim3 g3((unsigned)(a.blocks_c * cdiv(cdiv(a.nto, a.tpb), 1 << a.tsub_log2)),
                  (unsigned)a.ni, (unsigned)a.nbank);
#define BLDP_NARROWT(FF, TT)                                                  \
  if ((TT) <= 2 && a.tpb == 4 / (TT))                                         \
    BLDP_LAUNCH((k_reduce_narrowt<OP, FF, TT, ((TT) <= 2 ? 4 : 16)>), g3, block, 0, s, a); \
  else if (a.tpb == 8 / (TT))                                                 \
    BLDP_LAUNCH((k_reduce_narrowt<OP, FF, TT, 8>), g3, block, 0, s, a);       \
  else                                                                        \
    BLDP_LAUNCH((k_reduce_narrowt<OP, FF, TT, 16>), g3, block, 0, s, a);
    if (a.F == 1 && a.T == 1) { BLDP_NARROWT(1, 1) }
    else if (a.F == 1 && a.T == 2) { BLDP_NARROWT(1, 2) }
    else if (a.F == 1 && a.T == 4) { BLDP_NARROWT(1, 4) }
    else if (a.F == 2 && a.T == 1) { BLDP_NARROWT(2, 1) }
    else if (a.F == 2 && a.T == 2) { BLDP_NARROWT(2, 2) }
    else if (a.F == 2 && a.T == 4) { BLDP_NARROWT(2, 4) }
    else if (a.F == 2 && a.T == 3) { BLDP_NARROWT(2, 3) }
    else return hipErrorInvalidValue;
#undef BLDP_NARROWT
    return hipGetLastError();
  }
  if (p.path == PATH_VEC && a.tpb > 1) {  // large groups, short time blocks: k_reduce_wavet
    constexpr int NW = 4 * 4;  // time blocks per batch x batches: see k_reduce_wavet
    (void)NW;
    const int64_t rw = (int64_t)a.tpb;  // time blocks per wave
    const dim3 g3((unsigned)(a.nco * cdiv(a.nto, 4 * rw)), (unsigned)a.ni, (unsigned)a.nbank);
    const unsigned wb = (unsigned)(a.nbank * a.nco);  // bpack: one wave per (bank, group)
    const dim3 g3b((unsigned)cdiv(a.nto, rw), (unsigned)a.ni, 1u);
#define BLDP_WAVETL(K, T)                                                        \
  if (a.bpack)                                                                   \
    BLDP_LAUNCH((k_reduce_wavet<OP, K, T, true>), g3b, dim3(64 * wb), 0, s, a);  \
  else                                                                           \
    BLDP_LAUNCH((k_reduce_wavet<OP, K, T, false>), g3, block, 0, s, a);          \
  break;
#define BLDP_WAVET_T(K)                      \
  switch (a.T) {                             \
    case 1: BLDP_WAVETL(K, 1)                \
    case 2: BLDP_WAVETL(K, 2)                \
    case 4: BLDP_WAVETL(K, 4)                \
    case 3: BLDP_WAVETL(K, 3)                \
    default: return hipErrorInvalidValue;    \
  }                                          \
  break;
    switch (a.k4) {
      case 2: BLDP_WAVET_T(2)
      case 4: BLDP_WAVET_T(4)
      case 8: BLDP_WAVET_T(8)
      case 16: BLDP_WAVET_T(16)
      default: return hipErrorInvalidValue;
    }
#undef BLDP_WAVET_T
#undef BLDP_WAVETL
    return hipGetLastError();
  }
  if (p.path == PATH_LANE && p.col3) {  // fqavby = 12, short time blocks: k_reduce_col3
    const dim3 g3((unsigned)(a.blocks_c * cdiv(a.nto, a.tpb)), (unsigned)a.ni, 1u);
    const dim3 b3(kCol3Threads);
    switch (a.T) {
      case 1: BLDP_LAUNCH((k_reduce_col3<OP, 1>), g3, b3, 0, s, a); break;
      case 2: BLDP_LAUNCH((k_reduce_col3<OP, 2>), g3, b3, 0, s, a); break;
      case 3: BLDP_LAUNCH((k_reduce_col3<OP, 3>), g3, b3, 0, s, a); break;
      case 4: BLDP_LAUNCH((k_reduce_col3<OP, 4>), g3, b3, 0, s, a); break;
      case 8: BLDP_LAUNCH((k_reduce_col3<OP, 8>), g3, b3, 0, s, a); break;
      default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
  }
  if (p.path == PATH_LANE && p.lanet) {  // short time blocks, small odd groups: k_reduce_lanet
    const dim3 g3(a.bpack ? (unsigned)(a.blocks_c * cdiv(a.nto, a.tpb))
                          : (unsigned)(a.blocks_c * cdiv(cdiv(a.nto, a.tpb), 1 << a.tsub_log2)),
                  (unsigned)a.ni, a.bpack ? 1u : (unsigned)a.nbank);
#define BLDP_LANETL(FF, TT)                                        \
  if (a.bpack)                                                     \
    BLDP_LAUNCH((k_reduce_lanes<OP, FF, TT>), g3, block, 0, s, a); \
  else                                                             \
    BLDP_LAUNCH((k_reduce_lanet<OP, FF, TT>), g3, block, 0, s, a); \
  break;
#define BLDP_LANET_T(FF)                   \
  switch (a.T) {                           \
    case 1: BLDP_LANETL(FF, 1)             \
    case 2: BLDP_LANETL(FF, 2)             \
    case 4: BLDP_LANETL(FF, 4)             \
    BLDP_T38_CASES(BLDP_LANETL, FF)        \
    default: return hipErrorInvalidValue;  \
  }                                        \
  break;
    switch (a.F) {
      case 3: BLDP_LANET_T(3)
      case 5: BLDP_LANET_T(5)
      case 6: BLDP_LANET_T(6)
      case 7: BLDP_LANET_T(7)
      case 12: BLDP_LANET_T(12)
      default: return hipErrorInvalidValue;
    }
#undef BLDP_LANET_T
#undef BLDP_LANETL
    return hipGetLastError();
  }
  if (p.path == PATH_VEC_ROW && a.tpb > 1) {  // short time blocks, several per workgroup
    const dim3 g3(a.bpack ? (unsigned)(a.blocks_c * cdiv(a.nto, a.tpb))
                          : (unsigned)(a.blocks_c * cdiv(cdiv(a.nto, a.tpb), 1 << a.tsub_log2)),
                  (unsigned)a.ni, (unsigned)(a.bpack ? a.nbank >> a.tsub_log2 : a.nbank));
#define BLDP_ROWTK(G, T, N)                                                \
  if (a.bpack)                                                             \
    BLDP_LAUNCH((k_reduce_rowt<OP, G, T, N, true>), g3, block, kRowtShm, s, a);   \
  else                                                                     \
    BLDP_LAUNCH((k_reduce_rowt<OP, G, T, N, false>), g3, block, kRowtShm, s, a);  \
  break;
#define BLDP_ROWTN(T, N)                                                                    \
  switch (a.F / 4) {                                                                        \
    case 1: BLDP_ROWTK(1, T, N)    \
    case 2: BLDP_ROWTK(2, T, N)    \
    case 4: BLDP_ROWTK(4, T, N)    \
    case 8: BLDP_ROWTK(8, T, N)    \
    case 16: BLDP_ROWTK(16, T, N)  \
    case 32: BLDP_ROWTK(32, T, N)  \
    case 64: BLDP_ROWTK(64, T, N)  \
    default: return hipErrorInvalidValue;                                                   \
  }
#define BLDP_ROWT(T)                 \
  if ((T) <= 2 && a.tpb == 4 / (T)) { \
    BLDP_ROWTN(T, ((T) <= 2 ? 4 : 8))  \
  } else if (a.tpb == 8 / (T)) {     \
    BLDP_ROWTN(T, 8)                 \
  } else if (a.tpb == 16 / (T)) {    \
    BLDP_ROWTN(T, 16)                \
  } else {                           \
    return hipErrorInvalidValue;     \
  }
#define BLDP_ROWTC(X, T) BLDP_ROWT(T) break;
    switch (a.T) {
      case 1: BLDP_ROWT(1) break;
      case 2: BLDP_ROWT(2) break;
      case 4: BLDP_ROWT(4) break;
      BLDP_T38_CASES(BLDP_ROWTC, 0)
      default: return hipErrorInvalidValue;
    }
#undef BLDP_ROWTC
#undef BLDP_ROWT
#undef BLDP_ROWTN
#undef BLDP_ROWTK
    return hipGetLastError();
  }
  if (p.path == PATH_VEC_ROW && a.rsplit > 1) {  // a block's rows over 2 / 4 slices
    const dim3 g3((unsigned)a.blocks_c, (unsigned)(a.ni * a.nto), (unsigned)a.nbank);
#define BLDP_ROWS(S)                                                                          \
  switch (a.F / 4) {                                                                          \
    case 1: BLDP_LAUNCH((k_reduce_rows<OP, 1, S>), g3, block, kRowShm, s, a); break;         \
    case 2: BLDP_LAUNCH((k_reduce_rows<OP, 2, S>), g3, block, kRowShm, s, a); break;         \
    case 4: BLDP_LAUNCH((k_reduce_rows<OP, 4, S>), g3, block, kRowShm, s, a); break;         \
    case 8: BLDP_LAUNCH((k_reduce_rows<OP, 8, S>), g3, block, kRowShm, s, a); break;         \
    case 16: BLDP_LAUNCH((k_reduce_rows<OP, 16, S>), g3, block, kRowShm, s, a); break;       \
    case 32: BLDP_LAUNCH((k_reduce_rows<OP, 32, S>), g3, block, kRowShm, s, a); break;       \
    case 64: BLDP_LAUNCH((k_reduce_rows<OP, 64, S>), g3, block, kRowShm, s, a); break;       \
    default: return hipErrorInvalidValue;                                                     \
  }
    if (a.rsplit == 2) {
      BLDP_ROWS(2)
    } else if (a.rsplit == 4) {
      BLDP_ROWS(4)
    } else {
      return hipErrorInvalidValue;
    }
#undef BLDP_ROWS
    return hipGetLastError();
  }
  if (p.path == PATH_VEC_ROW) {
    const dim3 g3((unsigned)a.blocks_c, (unsigned)(a.ni * a.nto), (unsigned)a.nbank);
    switch (a.F / 4) {
      case 1: BLDP_LAUNCH((k_reduce_row<OP, 1>), g3, block, kRowShm, s, a); break;
      case 2: BLDP_LAUNCH((k_reduce_row<OP, 2>), g3, block, kRowShm, s, a); break;
      case 4: BLDP_LAUNCH((k_reduce_row<OP, 4>), g3, block, kRowShm, s, a); break;
      case 8: BLDP_LAUNCH((k_reduce_row<OP, 8>), g3, block, kRowShm, s, a); break;
      case 16: BLDP_LAUNCH((k_reduce_row<OP, 16>), g3, block, kRowShm, s, a); break;
      case 32: BLDP_LAUNCH((k_reduce_row<OP, 32>), g3, block, kRowShm, s, a); break;
      case 64: BLDP_LAUNCH((k_reduce_row<OP, 64>), g3, block, kRowShm, s, a); break;
      default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
  }
  if (p.path == PATH_VEC_IL) {
    const dim3 g3((unsigned)a.blocks_c, (unsigned)(a.ni * a.nto), (unsigned)a.nbank);
    switch (a.k4) {
      case 2: BLDP_LAUNCH((k_reduce_il<OP, 2, il_gpw(2)>), g3, block, kIlShm, s, a); break;
      case 4: BLDP_LAUNCH((k_reduce_il<OP, 4, kIlGpw>), g3, block, kIlShm, s, a); break;
      case 8: BLDP_LAUNCH((k_reduce_il<OP, 8, kIlGpw>), g3, block, kIlShm, s, a); break;
      case 16: BLDP_LAUNCH((k_reduce_il<OP, 16, kIlGpw>), g3, block, kIlShm, s, a); break;
      default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
  } else if (p.path == PATH_VEC) {
    e = launch_vec<OP>(a, p, s);
  } else if (p.path == PATH_NARROW) {
    if (a.F == 1)
      BLDP_LAUNCH((k_reduce_narrow<OP, 1>), grid, block, kNarrowShm, s, a);
    else
      BLDP_LAUNCH((k_reduce_narrow<OP, 2>), grid, block, kNarrowShm, s, a);
    e = hipGetLastError();
  } else if (p.path == PATH_NARROW_MIS) {
    BLDP_LAUNCH((k_reduce_narrow_mis<OP, 1>), grid, block, 0, s, a);
    e = hipGetLastError();
  } else if (p.path == PATH_LANE) {
    switch (a.F) {
      case 2: BLDP_LAUNCH((k_reduce_lane<OP, 2>), grid, block, 0, s, a); break;
      case 3: BLDP_LAUNCH((k_reduce_lane<OP, 3>), grid, block, 0, s, a); break;
      case 5: BLDP_LAUNCH((k_reduce_lane<OP, 5>), grid, block, 0, s, a); break;
      case 6: BLDP_LAUNCH((k_reduce_lane<OP, 6>), grid, block, 0, s, a); break;
      case 7: BLDP_LAUNCH((k_reduce_lane<OP, 7>), grid, block, 0, s, a); break;
      default: return hipErrorInvalidValue;
    }
    e = hipGetLastError();
  } else if (p.path == PATH_TILE) {
    if (a.in_cs == 1)
      BLDP_LAUNCH((k_reduce_tile<OP, true>), grid, block, 0, s, a);
    else
      BLDP_LAUNCH((k_reduce_tile<OP, false>), grid, block, 0, s, a);
    e = hipGetLastError();
  } else {
    BLDP_LAUNCH((k_reduce_scalar<OP>), grid, block, 0, s, a);
    e = hipGetLastError();
  }
  if (e != hipSuccess || a.nchunk == 1) return e;
  const int64_t nout = (int64_t)a.nbank * a.nto * a.ni * a.nco;
  if (a.nchunk > 16) {
    const unsigned fg = (unsigned)std::min<int64_t>(cdiv(nout, 4), 16384);
    BLDP_LAUNCH((k_reduce_finalize_w<OP>), dim3(fg), block, 0, s, a);
  } else {
    const unsigned fg = (unsigned)std::min<int64_t>(cdiv(nout, kBlock), 8192);
    BLDP_LAUNCH((k_reduce_finalize<OP>), dim3(fg), block, 0, s, a);
  }
  return hipGetLastError();
}

}  // namespace

// ---------------------------------------------------------------------------

namespace {
// name, default, and what it selects (the defaults are the measured choices;
// each of them cites its A/B where the planner uses it)
struct PlanOptDef {
  const char *name;
  int64_t def;
  int64_t lo, hi;  // the values bldp_plan_option accepts (and -1: the default)
};
const PlanOptDef kPlanOpts[OPT_COUNT] = {
    {"row_split", -1, 1, 4},      // k_reduce_row's block over 1 / 2 / 4 workgroup slices; -1 by launch size
    {"ts_fill", 1, 0, 1},         // narrow vector-path windows split time over idle waves
    {"narrow_mis", 1, 0, 1},      // misaligned F = 1 on k_reduce_narrow_mis
    {"t38", 1, 0, 1},             // tavby = 3, 8 on the short-time-block kernels
    {"wide_split", 1, 0, 1},      // groups > 4096 channels split time by work, not rows
    {"narrow_tpb", 2, 0, 2},      // k_reduce_narrowt: 2 = incl. the copy, 1 = not it, 0 = off
    {"lane", 1, 0, 1},            // k_reduce_lane where the tile path cannot run
    {"lane3", 1, 0, 1},           // fqavby = 3 on the lane kernel everywhere
    {"lanet", 1, 0, 1},           // k_reduce_lanet for small odd groups, short time blocks
    {"lanet_pack", 1, 0, 1},      // narrow lanet windows: 2 / 4 time groups per workgroup
    {"vec_il", 1, 0, 1},          // k_reduce_il for F = 512 .. 4096
    {"vec_row", 1, 0, 1},         // k_reduce_row for F = 4 .. 256
    {"row_tpb", 1, 0, 1},         // k_reduce_rowt for short time blocks
    {"rowt_pack", 1, 0, 1},       // narrow rowt windows: 2 / 4 time groups per workgroup
    // rowt/narrowt: launches below this many workgroups per CU take 8 (4 at T <= 2) rows
    {"rowt_small", 64, 0, 1 << 20},
    {"wavet", 1, 0, 1},           // k_reduce_wavet where il is a poor fit
    {"unaligned_vec", 2, 0, 2},   // dword-aligned 16-byte loads: 1 = reduce, 2 = + kurtosis
    {"kurt_exact", 1, 0, 1},      // k_kurt_regs exact-count forms for 16 / 32 spectra
    {"kurt_mid_cpl", 2, 1, 2},    // 2: k_kurt_mid2 (two channels per lane) where it applies
    {"kurt_mid_small", 1, 0, 1},  // k_kurt_mid2 on 4 waves for <= 64 spectra
    // leaf plans below this many waves per CU: one channel per lane
    {"kurt_leaf_narrow", 4, 0, 1 << 20},
    {"kurt_leaf_tile", 1, 0, 1},  // k_kurt_tile for narrow short leaves
    {"typed_vec", 1, 0, 1},       // order-free typed reductions on k_reduce_typed_vec
    {"typed_kurt", 1, 0, 3},      // 8-bit getkurtosis from exact integer power sums (k_kurt_i8):
                                  // 1 4- or 8-byte words a lane by the plan's rule, 2 / 3 forced
    {"row_bpack", 1, 0, 1},       // k_reduce_rowt: lane sets over consecutive banks on narrow stitched rows
    {"lane_bpack", 1, 0, 1},      // k_reduce_lanes: lanet's lanes along narrow stitched band rows
    {"wave_bpack", 1, 0, 1},      // k_reduce_wavet: a wave per (bank, group) of <= 16-group stitched rows
    {"col3", 1, 0, 1},            // fqavby = 12, short time blocks: k_reduce_col3 (float4 columns)
    {"rowt_narrow8", 1, 0, 1},    // k_reduce_rowt: 8 rows per lane on <= 128-column windows too
    {"st_plain", 1, 0, 2},        // row / il stores: 0 always nt, 1 plain below 2 GB of traffic, 2 always plain
};
struct PlanOpts {
  std::atomic<int64_t> v[OPT_COUNT];  // -1 = no override
  PlanOpts() {
    for (auto &x : v) x.store(-1);
  }
} g_plan_opt;
}  // namespace

int64_t plan_opt(int k) {
  const int64_t v = g_plan_opt.v[k].load(std::memory_order_relaxed);
  return v >= 0 ? v : kPlanOpts[k].def;
}
int plan_opt_index(const char *name) {
  for (int k = 0; k < OPT_COUNT; ++k)
    if (std::strcmp(name, kPlanOpts[k].name) == 0) return k;
  return -1;
}
int64_t plan_opt_override(int k) { return g_plan_opt.v[k].load(std::memory_order_relaxed); }
bool plan_opt_valid(int k, int64_t v) {
  if (v < 0) return true;
  if (v < kPlanOpts[k].lo || v > kPlanOpts[k].hi) return false;
  return k != OPT_ROW_SPLIT || v == 1 || v == 2 || v == 4;
}
void plan_opt_domain(int k, int64_t *lo, int64_t *hi) {
  *lo = kPlanOpts[k].lo;
  *hi = kPlanOpts[k].hi;
}
void plan_opt_set(int k, int64_t v) { g_plan_opt.v[k].store(v, std::memory_order_relaxed); }

// Where the per-XCD tile order pays (the rule and its measurements: the
// comment above kIlXcdMinT).  `bytes`: the launch's algorithmic traffic.
bool xcd_order_pays(int path, const RedArgs &a, int64_t F, int64_t T, int64_t bytes) {
  const int64_t pitch = 4 * a.in_ld_t;  // bytes between a column's rows
  switch (path) {
    case PATH_VEC_IL: return T >= kIlXcdMinT && pitch <= kIlXcdMaxPitch;
    case PATH_VEC_ROW:
      if (a.tpb > 1) return bytes >= kRowtXcdBytes && pitch >= kRowXcdMinPitch;  // rowt
      return T >= kIlXcdMinT && pitch >= kRowXcdMinPitch && pitch <= kIlXcdMaxPitch;  // row(s)
    case PATH_NARROW:
      if (a.tpb > 1) return F == 2 && bytes >= kRowtXcdBytes;  // narrowt
      return true;  // narrow
    case PATH_VEC:
      if (a.tpb > 1) return false;  // wavet
      return true;  // vec
    case PATH_TILE: return false;
    default: return false;
  }
}

Plan plan_reduce(RedArgs &a, bool aligned, bool rows16, bool words, int num_cus, int xcd_lg) {
  Plan p{};
  const int64_t F = a.F, T = a.T;
  p.nout = a.nco * a.ni * a.nto;
  const int64_t target_waves = (int64_t)num_cus * 16;  // ~4 waves per SIMD
  int64_t tiles;  // independent wave/thread tiles before any time split
  a.ts = 1;
  a.k4 = 1;
  a.tpb = 1;
  a.tsub_log2 = 0;
  a.rsplit = 1;
  a.bpack = 0;
  a.st_plain = 0;
  const bool t38 = opt(OPT_T38) != 0;
  if (opt(OPT_LANET) && words && a.in_cs == 1 && (T == 1 || T == 2 || T == 4 || (t38 && (T == 3 || T == 8))) &&
      (F == 3 || F == 5 || F == 6 || F == 7 || F == 12) && a.ni <= 65535 && a.nbank <= 65535 &&
      cdiv(a.nco + lanet_oalign_pad(), (int64_t)kBlock) * cdiv(a.nto, kLanetRows / T) <=
          INT32_MAX) {
    // small odd groups, short time blocks: one lane per group, NRW rows per lane
    p.path = PATH_LANE;
    p.lanet = true;
    a.tpb = (int32_t)(kLanetRows / T);
    a.blocks_c = cdiv(a.nco + lanet_oalign_pad(), (int64_t)kBlock);
    // narrow windows: 2 or 4 time groups per workgroup (the 0001 product at
    // fqavby = 12: 42 groups a row kept 42 of 256 lanes busy)
    if (opt(OPT_LANET_PACK))
      a.tsub_log2 = a.nco + 15 <= 64 ? 2 : a.nco + 15 <= 128 ? 1 : 0;
    a.nchunk = 1;
    a.rows_per_chunk = T;
    a.ntiles = a.blocks_c * cdiv(cdiv(a.nto, a.tpb), (int64_t)1 << a.tsub_log2) * a.ni * a.nbank;
    // a stitched band of banks narrower than a workgroup: lanes along the
    // product row (k_reduce_lanes, option lane_bpack)
    const int64_t row = a.nbank * a.nco;
    // (F = 12: 2.94 vs 2.90 ms on the 0001 band, not taken; F = 3 3.53 vs
    // 4.21, profiles/r04/ab_t1_0001_r04h.json)
    // (T <= 4: at T = 8, 2% slower on the 0001 band)
    if (opt(OPT_LANE_BPACK) && F <= 7 && T <= 4 && a.nbank > 1 && a.out_bank == a.nco &&
        a.nco + 15 < kBlock &&
        row <= UINT32_MAX - kBlock && cdiv(row, (int64_t)kBlock) * cdiv(a.nto, a.tpb) <= INT32_MAX) {
      a.bpack = 1;
      a.tsub_log2 = 0;
      a.blocks_c = cdiv(row, (int64_t)kBlock);
      a.ntiles = a.blocks_c * cdiv(a.nto, a.tpb) * a.ni;
    }
    // fqavby = 12: float4 columns, three lanes a group (k_reduce_col3, option
    // col3); any output layout, several banks per workgroup
    // (rows of < 65536 groups: the 0000 product's 5.6M-group rows lost 3-5% at
    // T = 2..4, profiles/r04/ab_grid0_r04l.json)
    if (opt(OPT_COL3) && F == 12 && (T == 1 || T == 2 || T == 3 || T == 4 || T == 8) &&
        a.nco < 65536 &&
        3 * a.nco * a.nbank <= UINT32_MAX - kCol3Threads &&
        cdiv(a.nbank * a.nco, (int64_t)64) * cdiv(a.nto, (int64_t)(4 / T > 0 ? 4 / T : 1)) <=
            INT32_MAX) {
      p.col3 = true;
      a.bpack = 0;
      a.tsub_log2 = 0;
      a.tpb = (int32_t)(4 / T > 0 ? 4 / T : 1);
      a.blocks_c = cdiv(a.nbank * a.nco, (int64_t)64);
      a.ntiles = a.blocks_c * cdiv(a.nto, (int64_t)a.tpb) * a.ni;
    }
    p.grid = a.ntiles;
    p.ws_bytes = 0;
    a.div = (float)(F * T);
    return p;
  }
  if (aligned && F % 4 == 0) {
    p.path = PATH_VEC;
    const int64_t g4 = F / 4;
    int lpg = 1;
    while (lpg < 64 && g4 % (2 * lpg) == 0) lpg *= 2;
    p.lpg = lpg;
    a.k4 = (int32_t)(g4 / lpg);
    const int64_t ctiles = cdiv(a.nco, 64 / lpg);
    tiles = ctiles * a.ni * a.nto * a.nbank;
    // rows a time-split wave needs at least: groups wider than the interleaved
    // kernel's (G4 > 1024: one wave reads K4 > 16 float4 per lane per row) have
    // enough work in one row (fqavby = 65536 at tavby = 8 was 272 waves)
    const int64_t tsrows = (opt(OPT_WIDE_SPLIT) && a.k4 > 16) ? 1 : 8;
    while (a.ts < 4 && tiles * a.ts < target_waves && T >= 2 * a.ts * tsrows) a.ts *= 2;
    // no idle waves: a workgroup holds 4/ts column tiles, so narrow windows
    // (fewer than 4 column tiles, e.g. the 512-channel 0001 product) split
    // their time rows over the spare waves instead
    if (opt(OPT_TS_FILL))
      while (a.ts < 4 && ctiles < 4 / a.ts && T >= 2 * a.ts * 8) a.ts *= 2;
    a.blocks_c = cdiv(ctiles, 4 / a.ts);
    tiles *= a.ts;
  } else if (aligned && (F == 1 || F == 2) && (a.nco * F) % 4 == 0) {
    p.path = PATH_NARROW;
    const int64_t nc4 = a.nco * F / 4;
    a.blocks_c = cdiv(nc4, kBlock);
    tiles = cdiv(nc4, 64) * a.ni * a.nto * a.nbank;
  } else if (words && a.in_cs == 1 && opt(OPT_LANE) >= 1 &&
             (F == 2 || F == 3 || F == 5 || F == 6 || F == 7) &&
             (!rows16 || (opt(OPT_LANE3) && F == 3))) {
    // small odd / not-multiple-of-4 groups: one lane per output
    p.path = PATH_LANE;
    a.blocks_c = cdiv(a.nco, kBlock);
    tiles = cdiv(a.nco, 64) * a.ni * a.nto * a.nbank;
  } else if (rows16 && a.in_cs == 1 && opt(OPT_NARROW_MIS) >= 1 && F == 1) {
    // misaligned start, time integration: aligned columns realigned by shuffle
    // (F = 2 on the same kernel lost to the tile path: 6.06 vs 5.83 ms on the
    // 0000 band at c0 = 2, profiles/r02/ab_tile_narrow_mis.json; removed in
    // round 5)
    p.path = PATH_NARROW_MIS;
    a.blocks_c = cdiv(a.nco * F, kMisSpan);
    tiles = a.blocks_c * 4 * a.ni * a.nto * a.nbank;
  } else if (rows16 && a.in_cs >= 1 && a.in_cs <= 8 && F <= (kSpan - 4) / a.in_cs + 1) {
    p.path = PATH_TILE;
    a.gpt = ((kSpan - 4) / a.in_cs + 1) / F;
    a.blocks_c = cdiv(a.nco, a.gpt);
    tiles = a.blocks_c * 4 * a.ni * a.nto * a.nbank;
  } else {
    p.path = PATH_SCALAR;
    a.blocks_c = cdiv(a.nco, kBlock);
    tiles = cdiv(a.nco, 64) * a.ni * a.nto * a.nbank;
  }
  // Long time blocks with too few tiles: split the T rows across workgroups.
  const int64_t rows_per_wave = cdiv(T, a.ts);
  // float4 per lane in a wave's rows (wide groups: K4 of them per row)
  const int64_t wave_work =
      rows_per_wave * ((opt(OPT_WIDE_SPLIT) && p.path == PATH_VEC && a.k4 > 16) ? a.k4 : 1);
  int64_t nchunk = 1;
  if (tiles > 0 && tiles < target_waves && wave_work >= 128) {  // (empty windows: no split)
    nchunk = std::min<int64_t>(cdiv(target_waves, tiles), wave_work / 64);
    nchunk = std::min<int64_t>(nchunk, rows_per_wave);
    nchunk = std::max<int64_t>(nchunk, 1);
  }
  a.rows_per_chunk = cdiv(T, nchunk);
  if (a.rows_per_chunk < 1) a.rows_per_chunk = 1;
  a.nchunk = (int32_t)std::max<int64_t>(1, cdiv(T, a.rows_per_chunk));
  p.ws_bytes = a.nchunk > 1 ? (size_t)a.nchunk * a.nbank * p.nout * sizeof(float) : 0;
  a.ntiles = a.blocks_c * a.ni * a.nchunk * a.nto * a.nbank;
  p.grid = std::min<int64_t>(a.ntiles, INT32_MAX);  // tiles beyond: grid-stride loop
  // large groups with short time blocks where the interleaved kernel is a
  // poor fit (few groups per row, or its 3-D grid too small): k_reduce_wavet
  // (path "vector", a.tpb = time blocks per wave)
  if (opt(OPT_WAVET) && p.path == PATH_VEC && p.lpg == 64 &&
      (a.k4 == 2 || a.k4 == 4 || a.k4 == 8 || a.k4 == 16) &&
      (T == 1 || T == 2 || T == 4 || (t38 && T == 3)) &&  // (T = 8: -8%, ab_t38_r03w)
      a.ts == 1 && a.nchunk == 1 &&
      (a.nco < 4 || a.ni * a.nto > 65535) && a.ni <= 65535 &&
      a.nbank <= 65535) {
    const int64_t tb = std::max<int64_t>(1, 16 / (T * a.k4)), rw = tb * (tb >= 2 ? 1 : 4);
    if (a.nco * cdiv(a.nto, 4 * rw) <= INT32_MAX) {
      a.tpb = (int32_t)rw;
      a.ntiles = a.nco * cdiv(a.nto, 4 * rw) * a.ni * a.nbank;
      // a stitched band whose product row is <= 16 groups: one workgroup per
      // RW spectra with a wave per (bank, group), whole rows stored (wave_bpack)
      if (opt(OPT_WAVE_BPACK) && a.nbank > 1 && a.nbank * a.nco <= 16 && a.out_bank == a.nco) {
        a.bpack = 1;
        a.ntiles = cdiv(a.nto, rw) * a.ni;
      }
      p.grid = a.ntiles;
    }
  }
  // whole-time-block tiles of 512..4096-channel groups: interleaved kernel
  // (3-D grid, so every dimension must fit)
  if (opt(OPT_VEC_IL) && p.path == PATH_VEC && p.lpg == 64 && a.tpb == 1 &&
      (a.k4 == 2 || a.k4 == 4 || a.k4 == 8 || a.k4 == 16) && a.ts == 1 && a.nchunk == 1 &&
      cdiv(a.nco, il_gpw(a.k4)) <= INT32_MAX && a.ni * a.nto <= 65535 && a.nbank <= 65535) {
    p.path = PATH_VEC_IL;
    a.blocks_c = cdiv(a.nco, il_gpw(a.k4));
    a.ntiles = a.blocks_c * a.ni * a.nto * a.nbank;
    p.grid = a.ntiles;
  }
  // small power-of-two groups, whole time block per tile, no time split:
  // the lean row kernel (3-D grid, so every dimension must fit)
  if (opt(OPT_VEC_ROW) && p.path == PATH_VEC && a.k4 == 1 && a.ts == 1 && a.nchunk == 1 &&
      F >= 4 && F <= 256 && (F & (F - 1)) == 0 && a.nbank <= 65535) {
    const int64_t bc = cdiv(a.nco * (F / 4), kBlock);
    // short time blocks: 16 / T of them per workgroup (k_reduce_rowt; grid x =
    // column blocks x time groups, so long 0001-product windows fit too)
    int64_t tpb = (T == 1 || T == 2 || T == 4 || (t38 && (T == 3 || T == 8))) ? 16 / T : 1;
    if (opt(OPT_ROW_TPB) && tpb > 1 && a.nto > 1 && bc * cdiv(a.nto, tpb) <= INT32_MAX &&
        a.ni <= 65535) {
      p.path = PATH_VEC_ROW;
      a.blocks_c = bc;
      // <= 128 float4 columns: 2 or 4 time groups per workgroup (>= 64 lanes each)
      const int64_t cols = a.nco * (F / 4);
      a.tsub_log2 = opt(OPT_ROWT_PACK) ? (cols <= 64 ? 2 : cols <= 128 ? 1 : 0) : 0;
      // small launches: 8 rows per lane (4 at T <= 2), more workgroups (option rowt_small);
      // at T = 8 that is one time block per workgroup, i.e. k_reduce_row, whose
      // 3-D grid must then hold (IF, time block) in y
      // windows of <= 128 float4 columns (the 0001 product) take 8 rows too at
      // T = 1 and at F >= 64 (option rowt_narrow8: 0001 band at T = 1, F = 4 / 8
      // / 16 / 64 +1.2..6%, F = 64 T = 2 / 4 +4.5 / 1.8%; F = 16 T = 2, F = 8 T = 2
      // and F = 4 T = 3 -1.7..4%: not taken; profiles/r04/ab_t1_0001_r04{j,k}.json,
      // ab_grid1_r04p.json)
      // Small launches at T <= 2 take 4 rows (0002 band T = 1 / 2, F = 4..256
      // +2..6%, profiles/r04/ab_grid_r04x.json; the narrow 0001 windows stay on
      // 8: 4 lost 2-5% there, ab_t1_0001_r04x.json)
      const bool small = bc * cdiv(cdiv(a.nto, tpb), (int64_t)1 << a.tsub_log2) * a.ni *
                             a.nbank < opt(OPT_ROWT_SMALL) * num_cus;
      if ((small || (opt(OPT_ROWT_NARROW8) && cols <= 128 && (T == 1 || F >= 64))) &&
          (8 / T > 1 || (bc <= INT32_MAX && a.ni * a.nto <= 65535)))
        tpb = small && T <= 2 ? 4 / T : 8 / T;
      if (tpb == 1) {  // k_reduce_row
        a.tpb = 1;
        a.tsub_log2 = 0;
        a.ntiles = bc * a.ni * a.nto * a.nbank;
      } else {
        a.tpb = (int32_t)tpb;
        a.ntiles = bc * cdiv(cdiv(a.nto, tpb), (int64_t)1 << a.tsub_log2) * a.ni * a.nbank;
        // a stitched band of narrow banks whose row segments are < 128 bytes
        // (the 0001 band at fqavby = 64: 32 bytes a bank): the lane sets take
        // consecutive banks instead of time groups, so each product row gets
        // whole segments of 2^tsub_log2 banks (option row_bpack)
        const int64_t sets = (int64_t)1 << a.tsub_log2;
        if (opt(OPT_ROW_BPACK) && a.tsub_log2 > 0 && cols == (kBlock >> a.tsub_log2) &&
            a.nbank % sets == 0 && a.out_bank == a.nco && 4 * a.nco < 128 &&
            bc * cdiv(a.nto, tpb) <= INT32_MAX) {
          a.bpack = 1;
          a.ntiles = bc * cdiv(a.nto, tpb) * a.ni * (a.nbank / sets);
        }
      }
      p.grid = a.ntiles;
    } else if (bc <= INT32_MAX && a.ni * a.nto <= 65535) {
      p.path = PATH_VEC_ROW;
      a.blocks_c = bc;
      a.ntiles = a.blocks_c * a.ni * a.nto * a.nbank;
      // launches of whole 16-row batches with < 64 tiles per CU: the block's
      // rows split over 4 slices of the workgroup (2 for F = 256, whose
      // slices each fold 64 columns), so that the launch does not end on a
      // partial round of 64 KiB tiles (profiles/r04/ab_rows_r04c.json: one to
      // eight 0002 files 5-11% faster; 0000 bands, 256+ tiles per CU, 9-27%
      // slower split)
      // (F >= 128: only below 16 tiles per CU, in 2 slices; the 0002 band at
      // F = 128 / 256, 34 tiles per CU, lost 3-5% split, profiles/r04/
      // ab_grid_r04l.json)
      int64_t S = plan_opt(OPT_ROW_SPLIT);
      if (T % 16 != 0)
        S = 1;
      else if (S < 0)
        S = F >= 128 ? (a.ntiles < (int64_t)16 * num_cus ? 2 : 1)
                     : (a.ntiles < (int64_t)64 * num_cus ? 4 : 1);
      if (S == 2 || S == 4) {
        a.rsplit = (int32_t)S;
        a.blocks_c = cdiv(a.nco * (F / 4), kBlock / S);
        a.ntiles = a.blocks_c * a.ni * a.nto * a.nbank;
      }
      p.grid = a.ntiles;
    }
  }
  // narrow path, short time blocks: k_reduce_narrowt (grid as k_reduce_rowt's)
  if (opt(OPT_NARROW_TPB) && p.path == PATH_NARROW && a.nchunk == 1 &&
      (T == 1 || T == 2 || T == 4 || (t38 && T == 3 && F == 2)) &&
      (opt(OPT_NARROW_TPB) >= 1 + (F == 1 && T == 1)) && a.nto > 1 && a.ni <= 65535 && a.nbank <= 65535) {
    const int64_t cols = a.nco * F / 4;
    const int sh = cols <= 64 ? 2 : cols <= 128 ? 1 : 0;
    // fewer rows per lane (instead of 16) on launches under rowt_small (64)
    // workgroups per CU and, at T = 1, on windows of <= 128 float4 columns: 8
    // (T = 3, 4) or 4 (T = 1, 2). 8 against 16: the 0002 band at F = 1 / 2,
    // T = 1..4 +5..12%, the 0001 band F = 1 / 2 T = 1 +7 / 3%; 4 against 8 at
    // T = 1, 2 another 2..8% (0002 / 0001 bands); the 0000 band keeps 16
    // (profiles/r04/ab_grid_r04{o,w}.json, ab_t1_0001_r04{o,w}.json)
    int64_t tpb = 16 / T;
    if ((a.blocks_c * cdiv(cdiv(a.nto, tpb), (int64_t)1 << sh) * a.ni * a.nbank <
             opt(OPT_ROWT_SMALL) * num_cus ||
         (opt(OPT_ROWT_NARROW8) && cols <= 128 && T == 1)) && 8 / T >= 1)
      tpb = T <= 2 ? 4 / T : 8 / T;
    const int64_t x = a.blocks_c * cdiv(cdiv(a.nto, tpb), (int64_t)1 << sh);
    if (x <= INT32_MAX) {
      a.tpb = (int32_t)tpb;
      a.tsub_log2 = sh;
      a.ntiles = x * a.ni * a.nbank;
      p.grid = a.ntiles;
    }
  }
  // narrow-path vector stores
  a.vec_out = 0;
  if (p.path == PATH_VEC_ROW && a.tpb > 1) {  // k_reduce_rowt's 16-byte row-segment stores
    const uintptr_t op = (uintptr_t)a.out;
    a.vec_out = (op % 16 == 0) && a.out_bank % 4 == 0 && a.out_ld_i % 4 == 0 &&
                a.out_ld_t % 4 == 0;
  }
  if (p.path == PATH_NARROW_MIS) {  // float4 (F = 1) / float2 (F = 2) stores at aligned co
    const int64_t w = 4 / F;            // outputs per lane
    const uintptr_t op = (uintptr_t)a.out;
    a.vec_out = (op % (4 * w) == 0) && a.out_bank % w == 0 && a.out_ld_i % w == 0 &&
                a.out_ld_t % w == 0;
  }
  if (p.path == PATH_NARROW) {
    const int64_t w = 4 / F;  // outputs per lane
    const uintptr_t op = (uintptr_t)a.out;
    a.vec_out = (op % (4 * w) == 0) && a.out_bank % w == 0 && a.out_ld_i % w == 0 &&
                a.out_ld_t % w == 0;
  }
  // output stores of the row / interleaved kernels: plain below 2 GB of
  // launch traffic, non-temporal above (option st_plain: 0 always nt, 1 (the
  // default) by that size rule, 2 always plain)
  {
    const int64_t bytes = 4 * a.nbank * a.ni * (a.nco * F * a.nto * T + a.nco * a.nto);
    const int64_t o = opt(OPT_ST_PLAIN);
    a.st_plain = o == 2 ? 1 : o == 0 ? 0 : (bytes < ((int64_t)2 << 30) ? 1 : 0);
    a.xcd_lg = xcd_order_pays(p.path, a, F, T, bytes) ? xcd_lg : 0;
  }
  a.div = (float)(F * T);
  return p;
}

void set_launch_events(hipEvent_t start, hipEvent_t stop) {
  t_ev_start = start;
  t_ev_stop = stop;
}

hipError_t launch_reduce(const RedArgs &a, const Plan &p, int op, hipStream_t s) {
  if (p.grid <= 0) return hipSuccess;
  switch (op) {
    case BLDP_OP_SUM: return launch_op<BLDP_OP_SUM>(a, p, s);
    case BLDP_OP_MEAN: return launch_op<BLDP_OP_MEAN>(a, p, s);
    case BLDP_OP_MAX: return launch_op<BLDP_OP_MAX>(a, p, s);
    case BLDP_OP_MIN: return launch_op<BLDP_OP_MIN>(a, p, s);
  }
  return hipErrorInvalidValue;
}

hipError_t launch_stitch(int nbank, const float *g, int64_t nc, int64_t nrows, float *out,
                         hipStream_t s) {
  const int64_t n = (int64_t)nbank * nc * nrows;
  if (n == 0) return hipSuccess;
  const bool v = nc % 4 == 0 && (uintptr_t)g % 16 == 0 && (uintptr_t)out % 16 == 0;
  const int64_t work = v ? n / 4 : n;
  const unsigned grid = (unsigned)std::min<int64_t>(cdiv(work, kBlock), 16384);
  if (v)
    hipLaunchKernelGGL(k_stitch4, dim3(grid), dim3(kBlock), 0, s, nbank, g, nc, nrows, out);
  else
    hipLaunchKernelGGL(k_stitch1, dim3(grid), dim3(kBlock), 0, s, nbank, g, nc, nrows, out);
  return hipGetLastError();
}

hipError_t launch_despike(float *d, int64_t nchan, int64_t nrows, int64_t nfpc, int64_t nspike,
                          hipStream_t s) {
  const int64_t n = nrows * nspike;
  if (n == 0) return hipSuccess;
  const unsigned grid = (unsigned)std::min<int64_t>(cdiv(n, kBlock), 16384);
  hipLaunchKernelGGL(k_despike, dim3(grid), dim3(kBlock), 0, s, d, nchan, nrows, nfpc, nspike);
  return hipGetLastError();
}

hipError_t launch_synth(float *out, int64_t nchan, int64_t nif, int64_t ntime, int64_t nfpc,
                        uint64_t seed, int kind, hipStream_t s) {
  const int64_t n = nchan * nif * ntime;
  if (n == 0) return hipSuccess;
  const int vec = ((uintptr_t)out % 16) == 0;
  const unsigned grid = (unsigned)std::min<int64_t>(cdiv(cdiv(n, 4), kBlock), 65536);
  hipLaunchKernelGGL(k_synth, dim3(grid), dim3(kBlock), 0, s, out, n, nchan, nfpc, seed, kind,
                     vec);
  return hipGetLastError();
}

}  // namespace bldp

// ---------------------------------------------------------------------------
// Window gather from decoded HDF5 chunks (the bitshuffle/LZ4 read path).
// The chunks covering the window are decoded back to back in chunk-grid
// order [gt][gi][gc] (each chunk C-order [ct][ci][cc]); this copies the
// window (nc, ni, nt) out of them into a dense Julia-order tensor.
namespace bldp {
namespace {
__global__ __launch_bounds__(256) void k_unchunk(const float *__restrict__ packed,
                                                 UnchunkArgs u, float *__restrict__ out) {
  const int64_t n = u.nc * u.ni * u.nt;
  const int64_t cvol = u.ct * u.ci * u.cc;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < n;
       e += (int64_t)gridDim.x * 256) {
    const int64_t c = e % u.nc, r = e / u.nc, i = r % u.ni, t = r / u.ni;
    // absolute dataset coordinates, then relative to the chunk bounding box
    const int64_t gc = u.c0 + c * u.cs - u.bc0, gi = u.i0 + i * u.is - u.bi0,
                  gt = u.t0 + t * u.ts - u.bt0;
    const int64_t kc = gc / u.cc, ki = gi / u.ci, kt = gt / u.ct;
    const int64_t slot = (kt * u.gi + ki) * u.gc + kc;
    out[e] = packed[slot * cvol + ((gt - kt * u.ct) * u.ci + (gi - ki * u.ci)) * u.cc +
                    (gc - kc * u.cc)];
  }
}
}  // namespace

hipError_t launch_unchunk(const float *packed, const UnchunkArgs &u, float *out, hipStream_t s) {
  const int64_t n = u.nc * u.ni * u.nt;
  if (n == 0) return hipSuccess;
  const unsigned grid = (unsigned)std::min<int64_t>((n + 255) / 256, 65536);
  hipLaunchKernelGGL(k_unchunk, dim3(grid), dim3(256), 0, s, packed, u, out);
  return hipGetLastError();
}
}  // namespace bldp
