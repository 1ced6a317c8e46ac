// Internal launch interface shared by kernels.hip and api.hip (not part of the ABI).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <mutex>
#include <vector>

#include "bldp.h"

namespace bldp {

// Record the thread-local error message returned by bldp_last_error; returns code.
int set_error(int code, const char *fmt, ...);

// Library-owned device scratch cached per (device, stream).  A lease keeps
// the (device, stream) entry locked until it is destroyed: take it before the
// first launch that uses the buffer and keep it until the last is queued, so
// host threads sharing a stream never interleave their kernels on it.
// Growing synchronizes that stream first.
struct ScratchLease {
  void *ptr = nullptr;
  std::unique_lock<std::mutex> hold;
};
int scratch_lease(hipStream_t s, size_t bytes, ScratchLease *lease);
// bldp_bslz4_decode_dev_async with chunk k's host header at comp_host +
// (chunk_off[k] - host_base) (bslz4.hip; the chunk reader's slot ring)
int bslz4_decode_async_at(int nchunk, const uint8_t *comp_host, uint64_t host_base,
                          const uint8_t *comp_dev, const uint64_t *chunk_off,
                          const uint64_t *chunk_len, int elem_size, uint8_t *out_dev,
                          const uint64_t *out_off, const uint64_t *out_len, int *err_dev,
                          hipStream_t s);
std::vector<int> scratch_devices();  // devices holding scratch
void scratch_release_all();          // frees it (callers drained the devices)
// The native file readers (fileio.hip): stop the reader threads and free the
// pinned slot ring (waits for a read call in progress).
void fileio_release();

// A host-staging pipeline (runtime.hip): two streams and four cached device
// buffers (slots 0/1 = input of stream 0/1, 2/3 = output of stream 0/1).
struct Stager {
  int dev = -1;
  hipStream_t st[2] = {nullptr, nullptr};
  void *buf[4] = {nullptr, nullptr, nullptr, nullptr};
  size_t bytes[4] = {0, 0, 0, 0};
  std::vector<void *> temp;  // oversize buffers of the current call
};
// Take an idle pipeline of `dev` (created on first use); the device must be gfx950.
int stager_acquire(int dev, Stager **out);
// Device buffer of >= need bytes for `slot`, valid until stager_release.
int stager_buffer(Stager *s, int slot, size_t need, void **p);
void stager_release(Stager *s);
// The library's persistent worker stream on `dev`.
int device_stream(int dev, hipStream_t *out);

// One reduction launch: nbank banks with identical geometry.
// Window element (c, i, t) of bank b sits at
//   in[b][in_off + c*in_cs + i*in_ld_i + t*in_ld_t]
// and output element (c', i, t') of bank b is written at
//   out[b*out_bank + c' + i*out_ld_i + t'*out_ld_t].
struct RedArgs {
  const float *in[BLDP_MAX_BANKS];
  float *out;
  float *ws;  // partials [nchunk][nbank][nto][ni][nco] when nchunk > 1
  int64_t out_bank, out_ld_i, out_ld_t;
  int64_t in_off, in_cs, in_ld_i, in_ld_t;
  int64_t nco, ni, nto, F, T;
  int64_t rows_per_chunk;  // time rows of one T-block handled by one block
  int64_t blocks_c;        // blocks along the output-channel axis
  int64_t ntiles;          // workgroup tiles (grid may be smaller: grid-stride)
  int32_t nchunk, nbank;
  int32_t ts;              // waves of a tile that split the T rows (1, 2, 4)
  int32_t k4;              // float4 loads per lane per row (vector path)
  int32_t vec_out;         // narrow path: 16/8-byte output stores are legal
  int64_t gpt;             // tile path: output channels (groups) per workgroup tile
  int32_t tpb;             // row path: time blocks per workgroup (k_reduce_rowt when > 1)
  int32_t tsub_log2;       // k_reduce_rowt: log2 of the time groups sharing a workgroup
  int32_t bpack;           // k_reduce_rowt: the 2^tsub_log2 lane sets take consecutive banks;
                           // lane path: k_reduce_lanes (lanes along the stitched row)
  int32_t rsplit;          // k_reduce_rows: slices of a workgroup splitting a block's rows (1 = k_reduce_row)
  int32_t st_plain;        // row / il / rowt output stores plain (1) or non-temporal (0)
  int32_t xcd_lg;          // log2 XCDs of the per-XCD tile order (xcd_order), 0 = off
  float div;               // F*T, the mean divisor
};

// Runtime plan options (bldp_plan_option): process-wide overrides of the
// planners' choices, for tests that enumerate every form of a plan and for
// A/B timing in one process.  plan_opt returns the override, or the option's
// default (the measured choice) when there is none; -1 = "the planner
// decides by shape" where an option has that setting (row_split).
// Names and defaults: kernels.hip kPlanOpts.
enum PlanOpt {
  OPT_ROW_SPLIT = 0, OPT_TS_FILL, OPT_NARROW_MIS, OPT_T38,
  OPT_WIDE_SPLIT, OPT_NARROW_TPB, OPT_LANE, OPT_LANE3, OPT_LANET, OPT_LANET_PACK, OPT_VEC_IL,
  OPT_VEC_ROW, OPT_ROW_TPB, OPT_ROWT_PACK, OPT_ROWT_SMALL, OPT_WAVET, OPT_UNALIGNED_VEC,
  OPT_KURT_EXACT, OPT_KURT_MID_CPL, OPT_KURT_MID_SMALL, OPT_KURT_LEAF_NARROW, OPT_KURT_LEAF_TILE,
  OPT_TYPED_VEC, OPT_TYPED_KURT, OPT_ROW_BPACK, OPT_LANE_BPACK, OPT_WAVE_BPACK, OPT_COL3, OPT_ROWT_NARROW8, OPT_ST_PLAIN, OPT_COUNT
};
int64_t plan_opt(int k);
inline int64_t opt(int k) { return plan_opt(k); }
// name -> option index, or -1
int plan_opt_index(const char *name);
int64_t plan_opt_override(int k);  // -1 = none
bool plan_opt_valid(int k, int64_t v);  // v in the option's domain (or < 0: the default)
void plan_opt_domain(int k, int64_t *lo, int64_t *hi);
void plan_opt_set(int k, int64_t v);

enum Path { PATH_VEC = 0, PATH_NARROW = 1, PATH_SCALAR = 2, PATH_TILE = 3, PATH_VEC_IL = 4,
            PATH_VEC_ROW = 5, PATH_NARROW_MIS = 6, PATH_LANE = 7 };

struct Plan {
  int path;
  int lpg;                   // lanes per output group (vector path)
  bool lanet;                // lane path: k_reduce_lanet (NRW rows per lane) not k_reduce_lane
  bool col3;                 // lane path at fqavby = 12: k_reduce_col3 (float4 columns)
  int64_t grid;             // blocks of 256 threads
  int64_t nout;              // outputs per bank
  size_t ws_bytes;           // partial workspace required (0 if nchunk == 1)
};

// Fill the launch geometry (path, lpg, ts, k4, nchunk, rows_per_chunk,
// blocks_c, grid) for an args struct whose shape/stride fields are set.
// `aligned` says whether 16-byte vector loads of every group are legal;
// `rows16` whether every bank pointer is 16-byte aligned and the IF/time
// pitches are multiples of 4 floats (any channel offset and step); `words`
// whether the channel step is 1 and every bank pointer is dword-aligned.
// xcd_lg: log2 of the device's XCD count (0: one XCD, or not a power of two)
Plan plan_reduce(RedArgs &a, bool aligned, bool rows16, bool words, int num_cus, int xcd_lg);

hipError_t launch_reduce(const RedArgs &a, const Plan &p, int op, hipStream_t s);
// events the next launch_reduce's dispatches carry (null, null: none)
void set_launch_events(hipEvent_t start, hipEvent_t stop);

hipError_t launch_stitch(int nbank, const float *g, int64_t nc, int64_t nrows, float *out,
                         hipStream_t s);
hipError_t launch_despike(float *d, int64_t nchan, int64_t nrows, int64_t nfpc, int64_t nspike,
                          hipStream_t s);

// Kurtosis launch (kurtosis.hip).  Julia's Float32 mean is a pairwise sum
// whose halving tree is perfect down to level K ("blocks", <= 2048 spectra),
// each block being one or two sequentially summed leaves (<= 1024 spectra).
struct KurtArgs {
  const float *in[BLDP_MAX_BANKS];  // banks with identical geometry
  int32_t nbank;
  int64_t nrow;                     // nbank * ni output rows of nc channels
  int64_t in_off, in_cs, in_ld_i, in_ld_t;
  int64_t nc, ni, nt;
  int32_t vec;  // float4 along channels legal
  int32_t rows16;  // ... and every float4 is 16-byte aligned (global_load_lds)
  int32_t K;    // level of the blocks of the pairwise-sum tree
  int64_t nslot;  // leaf slots, 2 per block (2^(K+1))
  int64_t nseg;   // 64-lane column segments per row (k_kurt_leaf)
  int32_t leafw;  // channels per lane of k_kurt_leaf (kLeafW; 1 for short narrow windows)
  int32_t leaftile;  // leaves read whole into registers: k_kurt_tile's lane groups per channel (0 = streamed)
  // two-pass (unaligned) z pass
  int64_t rows_per_chunk;
  int32_t nchunk;
  int32_t ts;       // waves of a workgroup splitting the spectra of a tile (1, 2, 4)
  float *mean;      // [nbank*ni][nc]  Float32 mean (two-pass path)
  double *ws_mom;   // [nchunk][2][nbank*ni][nc]
  // leaf / tree-node partials: pm [4][nodes][n] Float64 (mean, M2, M3, M4
  // about the node's own mean), pf [3][nodes][n] Float32 (pairwise sum, max, min)
  double *pm;
  float *pf;
  double *out;      // [nbank][ni][nc]
};
void plan_kurtosis(KurtArgs &k, int num_cus);
size_t kurtosis_ws_bytes(const KurtArgs &k);
hipError_t launch_kurtosis(KurtArgs &k, char *ws, hipStream_t s);
// Which kurtosis path a plan takes (0 registers, 1 register tile, 2 streamed
// leaves + tree merge, 3 two passes), for tests and bench.
int kurtosis_path(const KurtArgs &k);
int64_t kurtosis_max_grid(const KurtArgs &k);  // largest grid of the plan

// Window of a chunked dataset: chunk dims (ct, ci, cc) in C order, a chunk
// bounding box starting at (bt0, bi0, bc0) with (gt, gi, gc) chunks, and the
// window {c0, nc, cs, i0, ni, is, t0, nt, ts} in dataset coordinates.
struct UnchunkArgs {
  int64_t ct, ci, cc, bt0, bi0, bc0, gt, gi, gc;
  int64_t c0, nc, cs, i0, ni, is, t0, nt, ts;
};
hipError_t launch_unchunk(const float *packed, const UnchunkArgs &u, float *out, hipStream_t s);

// Reductions and kurtosis of non-Float32 elements (typed.hip).  Element
// (c, i, t) of bank b at in[b][in_off + c*in_cs + i*in_ld_i + t*in_ld_t],
// output (c', i, t') at out[b*out_bank + c' + i*out_ld_i + t'*out_ld_t]
// (kurtosis: out dense [nbank][ni][nco], nto = the spectra).
struct TypedArgs {
  const void *in[BLDP_MAX_BANKS];
  void *out;
  int32_t dtype, nbank;
  int64_t out_bank, out_ld_i, out_ld_t;
  int64_t in_off, in_cs, in_ld_i, in_ld_t;
  int64_t nco, ni, nto, F, T;
  int32_t num_cus;  // of the launch's device (the coalesced kernel's grid)
  void *ws;         // typed kurtosis: kurtosis_typed_ws_bytes of scratch (or null)
  size_t ws_bytes;  // its size (the launch re-plans and checks it: plan options are
                    // process-wide, so another thread may change them in between)
};
size_t dtype_size(int dtype);              // 0 = unknown
int typed_out_dtype(int dtype, int op);    // -1 = invalid
hipError_t launch_reduce_typed(const TypedArgs &a, int op, hipStream_t s);
hipError_t launch_kurtosis_typed(const TypedArgs &a, double *out, hipStream_t s);
size_t kurtosis_typed_ws_bytes(const TypedArgs &a);  // scratch launch_kurtosis_typed wants

hipError_t launch_synth(float *out, int64_t nchan, int64_t nif, int64_t ntime, int64_t nfpc,
                        uint64_t seed, int kind, hipStream_t s);

}  // namespace bldp
