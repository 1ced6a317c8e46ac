/*
 * bldp.h — C ABI of libbldp_hip, the MI355X engine for the worker-side
 * reduction of BLDistributedDataProducts.jl (reference v0.3.2).
 *
 * Every entry point here replaces one piece of the reference's Julia hot path
 * (paths are relative to the reference repo root):
 *
 *   bldp_reduce_f32        fqav(A, n; f) src/gbtworkerfunctions.jl:16-20, applied
 *                          to the window read at :182-186 / :173-174, plus the
 *                          additive time integration (fqav on axis 3).
 *   bldp_reduce_host_f32   same, for a host array (what WorkerFunctions.getdata
 *                          holds after the HDF5/mmap read, :174 / :188).
 *   bldp_band_reduce_f32   GBT.getdata fan-out (src/gbt.jl:69-79) + the band
 *                          stitch reduce(vcat, ...) (src/gbt.jl:103) for banks
 *                          resident on one GPU.
 *   bldp_stitch_f32        reduce(vcat, banks) (src/gbt.jl:103) of bank-major
 *                          gathered blocks.
 *   bldp_comm_* /          GBT.getdata's fetch of every worker's result to the
 *   bldp_band_gather_f32   caller (src/gbt.jl:75-78) as an RCCL gather over xGMI.
 *   bldp_despike_f32       d[spike:nfpc:end,:,:] .= d[spike-1:nfpc:end,:,:]
 *                          (src/gbt.jl:101-102,111).
 *   bldp_kurtosis_f32      getkurtosis (src/gbtworkerfunctions.jl:197-202) with
 *                          StatsBase.kurtosis' two-pass recipe.
 *   bldp_fqav_range        fqav(r::AbstractRange, n) src/gbtworkerfunctions.jl:27-33.
 *   bldp_bslz4_*           HDF5 filter 32008 decode behind h5["data"][idxs...]
 *                          (:181-187; H5Zbitshuffle, Project.toml:10).
 *
 * Conventions
 *   - Arrays are Julia column-major (nchan, nif, ntime), channel fastest
 *     (README.md:165-168); in C terms data[t][i][c].
 *   - A window is 9 int64: {c0, nc, cs, i0, ni, is, t0, nt, ts} = 0-based
 *     start, count and step per axis (a Julia range a:s:b becomes start=a-1,
 *     count=length, step=s).  NULL means the whole array, i.e. idxs=(:,:,:).
 *   - fqavby <= 1 / tavby <= 1 disable that axis (fqav returns A, :17).
 *     fqavby must divide nc (Julia reshape -> DimensionMismatch, :18-19);
 *     tavby must divide nt (same rule on axis 3).  Both give BLDP_EDIM.
 *   - "_f32" device entry points take DEVICE pointers and a hipStream_t passed
 *     as void* (NULL = the null stream).  They are asynchronous on that stream
 *     and never synchronize; buffers are owned by the caller.
 *   - Return value 0 = ok, negative = error; bldp_last_error() returns the
 *     thread-local message of the last failing call.
 *
 * Threading ("reentrant per device handle")
 *   - Every entry point may be called from several host threads at once, for
 *     the same or different devices (GBT.getdata's per-worker fan-out,
 *     src/gbt.jl:75-77).  Library state shared between calls (per-(device,
 *     stream) scratch, staging pipelines, pinned slot rings, reader threads)
 *     is leased per call under its own lock; results never depend on what
 *     another thread is doing.
 *   - The only process-wide mutable setting is bldp_plan_option, an A/B and
 *     test facility: the product path never sets it, and a caller that sets
 *     it changes the kernel choice (never the results: every form is
 *     bit-identical or held to the same tolerance) of every thread's later
 *     plans.  Choices that are part of a call (e.g. the staged branch of
 *     bldp_band_reduce_multi_f32) are arguments of that call.
 *   - Asynchronous entry points order their work on the caller's stream only;
 *     a caller that hands data between streams or threads does the ordering
 *     (events) itself.
 */
#ifndef BLDP_H
#define BLDP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 2: bldp_bslz4_decode_dev / _async take out_len (round 2); BLDP_EIO; the
 *    typed (non-Float32) entry points
 * 3: prepared band reduces (bldp_band_reduce_prepare_f32 / bldp_reduce_launch /
 *    bldp_reduce_launch_timed / bldp_reduce_release); bldp_plan_option; bldp_file_runs_to_device
 * 4: bldp_band_reduce_multi_f32 takes a flags word (BLDP_BAND_STAGED replaces
 *    the process-wide "force_staged" option and BLDP_FORCE_STAGED);
 *    bldp_peer_access; bldp_device_to_host; bldp_file_chunks_to_device;
 *    bldp_chunks_to_device stages through the pinned slot ring when
 *    host_pinned is NULL;
 *    bldp_plan_option checks each
 *    option's domain; bldp_read_probe moved out of the product library
 *    (tools/hbm_probe.hip, build/libbldp_probe.so); plan options
 *    "force_staged", "il_persist", "max_wg_per_cu", "typed_rows" removed, and
 *    the values that only ever forced a losing form (narrow_mis 2, lane 2,
 *    wavet 2, unaligned_vec 3, kurt_leaf_tile 2)
 * 5: bldp_reduce_prepare / bldp_kurtosis_prepare (any element type) launched
 *    by bldp_reduce_launch; bldp_band_reduce_multi_f32 flag
 *    BLDP_BAND_PEER_STORE (direct xGMI stores are opt-in); plan option
 *    "typed_kurt" */
#define BLDP_ABI_VERSION 5

#if defined(BLDP_BUILD)
#define BLDP_API __attribute__((visibility("default")))
#else
#define BLDP_API
#endif

/* fqavfunc values named by README.md:192-195 */
enum bldp_op { BLDP_OP_SUM = 0, BLDP_OP_MEAN = 1, BLDP_OP_MAX = 2, BLDP_OP_MIN = 3 };

/* error codes */
#define BLDP_OK 0
#define BLDP_EINVAL (-1)  /* bad argument / AssertionError analogue            */
#define BLDP_EDIM (-2)    /* DimensionMismatch: fqavby/tavby does not divide     */
#define BLDP_EHIP (-3)    /* HIP runtime error                                   */
#define BLDP_ENOMEM (-5)  /* device or pinned allocation failed                  */
#define BLDP_EBOUNDS (-6) /* window outside the array (BoundsError analogue)     */
#define BLDP_ECOMM (-7)   /* RCCL error in the cross-GPU band exchange          */
#define BLDP_EIO (-8)     /* a file read failed or ended early (truncated file)  */

#define BLDP_MAX_BANKS 64

BLDP_API int bldp_abi_version(void);
/* Copy the last error message of this thread into buf (NUL-terminated). */
BLDP_API int bldp_last_error(char *buf, size_t len);
/* Number of visible GPUs. */
BLDP_API int bldp_device_count(int *n);

/* Library setup (SURVEY §8 B2 bldp_init/bldp_finalize; called where the
 * reference sets up its workers, GBT.setupworkers, src/gbt.jl:12-46).
 * devs == NULL selects every visible device.  Checks each device is gfx950
 * (BLDP_EINVAL otherwise), creates its worker stream and one warm
 * host-staging pipeline, and enables peer access between the listed devices.
 * Optional: every entry point initialises what it needs on first use. */
BLDP_API int bldp_init(int ndev, const int *devs);
/* Drain the devices and free every library-owned resource (scratch,
 * staging pipelines, streams).  BLDP_EINVAL while a host call is running.
 * Later calls re-initialise lazily. */
BLDP_API int bldp_finalize(void);
/* Page-lock / unlock a long-lived caller host buffer so the host-array entry
 * points copy from it at full PCIe rate (hipHostRegister). */
BLDP_API int bldp_host_register(void *ptr, size_t bytes);
BLDP_API int bldp_host_unregister(void *ptr);

/* Output shape of a reduction: nco = nc/F, nto = nt/T (after the divisibility
 * checks), ni = window IF count.  Pure host function. */
BLDP_API int bldp_reduce_shape(int64_t nchan, int64_t nif, int64_t ntime, const int64_t *win,
                      int64_t fqavby, int64_t tavby, int64_t out_shape[3]);

/* Introspection (tests/bench): the launch plan bldp_reduce_f32 would use for
 * these pointers.  info = {path (0 vector, 1 narrow, 2 scalar, 3 tile,
 * 4 interleaved, 5 row, 6 narrow_mis, 7 lane), lanes per group, waves (row
 * path: workgroup slices) splitting T, float4 per lane per row, time chunks,
 * workgroups, workspace bytes, vector output stores}.  Launches nothing. */
BLDP_API int bldp_reduce_plan_f32(const float *in, int64_t nchan, int64_t nif, int64_t ntime,
                         const int64_t *win, int64_t fqavby, int64_t tavby, int op,
                         const float *out, int64_t info[8]);

/* Process-wide plan options, an A/B and TEST facility only (see Threading
 * above: the product path never sets one): override one of the planners'
 * measured choices.  value -1 restores the default; *previous (may be NULL)
 * receives the old override (-1 = none).  Every form is parity-tested
 * (tests/test_gpu_parity.py::test_plan_options_every_form).
 *   "row_split"      k_reduce_row's time block over 1, 2 or 4 slices of a
 *                    workgroup (whole 16-row batches only; bit-identical
 *                    forms); default -1 = chosen by launch size
 *   "ts_fill", "narrow_mis", "t38", "wide_split",
 *   "narrow_tpb", "lane", "lane3", "lanet", "lanet_pack", "vec_il",
 *   "vec_row", "row_tpb", "rowt_pack", "rowt_small", "wavet",
 *   "unaligned_vec", "kurt_exact", "kurt_mid_cpl", "kurt_mid_small",
 *   "kurt_leaf_narrow", "kurt_leaf_tile", "typed_vec", "typed_kurt",
 *   "row_bpack", "lane_bpack", "wave_bpack", "col3", "rowt_narrow8", "st_plain"
 *                    which kernel a reduce / kurtosis / typed shape takes
 *                    (csrc/kernels.hip kPlanOpts: defaults, meanings and the
 *                    values each option accepts).
 * Unknown names, and values outside an option's domain: BLDP_EINVAL. */
BLDP_API int bldp_plan_option(const char *name, int64_t value, int64_t *previous);

/* out[c', i, t'] = op over the F x T block of the window (device pointers).
 * out is dense (nco, ni, nto). */
BLDP_API int bldp_reduce_f32(const float *in, int64_t nchan, int64_t nif, int64_t ntime,
                    const int64_t *win, int64_t fqavby, int64_t tavby, int op, float *out,
                    void *stream);

/* Same with an explicit output layout: element (c', i, t') is written at
 * out[c' + out_ld_i * i + out_ld_t * t'] (lets a bank write straight into
 * its slot of a stitched band product). */
BLDP_API int bldp_reduce_strided_f32(const float *in, int64_t nchan, int64_t nif, int64_t ntime,
                            const int64_t *win, int64_t fqavby, int64_t tavby, int op,
                            float *out, int64_t out_ld_i, int64_t out_ld_t, void *stream);

/* Host-pointer form: in and out are host memory; the window is streamed to
 * device `dev` through double-buffered staging and reduced there.
 * Synchronous (returns when out is filled). */
BLDP_API int bldp_reduce_host_f32(int dev, const float *in, int64_t nchan, int64_t nif, int64_t ntime,
                         const int64_t *win, int64_t fqavby, int64_t tavby, int op, float *out);

/* Band of nbank banks on ONE device, all with the same (nchan, nif, ntime)
 * and window: reduces every bank and writes the stitched product
 * out (nbank*nco, ni, nto) in bank order, i.e. reduce(vcat, ...) of the
 * per-bank results (src/gbt.jl:103).  in[] is a HOST array of device
 * pointers.  One launch covers every bank. */
BLDP_API int bldp_band_reduce_f32(int nbank, const float *const *in, int64_t nchan, int64_t nif,
                         int64_t ntime, const int64_t *win, int64_t fqavby, int64_t tavby,
                         int op, float *out, void *stream);

/* bldp_band_reduce_f32 prepared once for fixed buffers: the argument checks,
 * window, launch plan and kernel arguments are computed here, so each
 * bldp_reduce_launch only queues the kernel(s) on `stream` (same results as
 * bldp_band_reduce_f32 with these arguments).  The handle is bound to the
 * current device and to these pointers; the caller keeps them alive until
 * bldp_reduce_release.  Same errors as bldp_band_reduce_f32 at prepare time;
 * a launch from another current device is BLDP_EINVAL. */
typedef struct bldp_reduce_op *bldp_reduce_op_t;
BLDP_API int bldp_band_reduce_prepare_f32(int nbank, const float *const *in, int64_t nchan,
                                          int64_t nif, int64_t ntime, const int64_t *win,
                                          int64_t fqavby, int64_t tavby, int op, float *out,
                                          bldp_reduce_op_t *handle);
BLDP_API int bldp_reduce_launch(bldp_reduce_op_t handle, void *stream);
/* bldp_reduce_launch with timing: the reduce's own kernel dispatches carry
 * the events (hipExtLaunchKernel), `ev_start` taking the first dispatch's
 * start and `ev_stop` the last one's end, so timing a launch queues nothing
 * between it and the next.  Both are hipEvent_t created with timing enabled;
 * read them with hipEventElapsedTime.  An empty reduce records neither. */
BLDP_API int bldp_reduce_launch_timed(bldp_reduce_op_t handle, void *stream, void *ev_start,
                                      void *ev_stop);
BLDP_API int bldp_reduce_release(bldp_reduce_op_t handle);

/* One process, one or more banks per GPU: bank b lives on
 * device bank_dev[b] (in[b] is a device pointer there).  Every device reduces
 * its banks into their vcat slots of `out`, the stitched (nbank*nco, ni, nto)
 * product on device `root`.  A device's banks are reduced by one launch per
 * run of evenly spaced bank indices (one launch per device for contiguous
 * shards).  The root's kernels store their slots directly; another device's
 * banks are reduced into library staging on that device and moved by one
 * strided peer copy per run (DMA over xGMI).  Synchronous; all banks share the
 * same (nchan, nif, ntime) and window.  Replaces the per-worker getdata +
 * reduce(vcat, ...) of GBT.getdata / loadscan (src/gbt.jl:75-78,103).
 * flags: 0, or one of
 *   BLDP_BAND_STAGED      every bank takes the staged branch, the root's banks
 *                         included (how a one-GPU box runs that branch);
 *   BLDP_BAND_PEER_STORE  devices with peer access to `root` store their
 *                         slots directly from the reduce kernels (xGMI
 *                         stores, no staging copy).  Opt-in: this branch has
 *                         not yet run on a multi-GPU node. */
#define BLDP_BAND_STAGED 1u
#define BLDP_BAND_PEER_STORE 2u
BLDP_API int bldp_band_reduce_multi_f32(int nbank, const int *bank_dev, const float *const *in,
                                        int64_t nchan, int64_t nif, int64_t ntime,
                                        const int64_t *win, int64_t fqavby, int64_t tavby,
                                        int op, int root, float *out, unsigned flags);

/* Whether kernels running on device `dev` may store straight into memory of
 * device `peer` (the same device, or peer access over xGMI, which this call
 * enables when the hardware allows it): *direct = 1, else 0 (the caller stages
 * and copies).  What GBT.getband's bank-by-bank branch asks before a bank's
 * reduce on its own GPU writes the root's vcat slot (src/gbt.jl:103). */
BLDP_API int bldp_peer_access(int dev, int peer, int *direct);

/* Device -> host copy of `bytes` from src (memory of the current device) into
 * ordinary (pageable) host memory dst through the library's ring of pinned
 * slots (the current device's, shared with the file readers): slot-sized DMA
 * copies on copy_stream, each landed slot copied out to dst by the reader
 * threads while the next DMA runs.  The copies start after the work queued so
 * far on `stream` (the producer's stream).  Synchronous: returns when dst is
 * filled.  No pinned memory is allocated per call, and dst is never
 * page-locked.  stats (NULL or 4 doubles): ms to the first DMA, total ms,
 * slots, copy-out threads. */
BLDP_API int bldp_device_to_host(const void *src, void *dst, int64_t bytes, void *copy_stream,
                                 void *stream, double *stats);

/* Band stitch across processes, one GPU each (the reference's one
 * Distributed.jl worker per bank, src/gbt.jl:75-77): an RCCL communicator
 * and ncclGather over xGMI (RCCL is loaded at run time).
 *   rank 0: bldp_comm_id(id), sends the 128 bytes to every rank;
 *   every rank: bldp_comm_init (collective), reduces its banks into a dense
 *   slice with bldp_band_reduce_f32, then bldp_band_gather_f32: the root's
 *   `gathered` receives nranks slices of `count` floats, rank-major;
 *   root: bldp_stitch_f32(nranks, gathered, ...) puts rank-major slices in
 *   vcat order (no-op layout when every bank's output is one (IF, time) row).
 * The gather is asynchronous on `stream`. */
#define BLDP_COMM_ID_BYTES 128
BLDP_API int bldp_comm_id(uint8_t id[BLDP_COMM_ID_BYTES]);
BLDP_API int bldp_comm_init(int dev, int nranks, int rank, const uint8_t id[BLDP_COMM_ID_BYTES],
                            void **comm);
BLDP_API int bldp_comm_destroy(void *comm);
BLDP_API int bldp_band_gather_f32(void *comm, int root, const float *slice, int64_t count,
                                  float *gathered, void *stream);

/* gathered: nbank dense blocks (nc, nif, ntime) back to back (bank-major,
 * what a gather to the root leaves); out: (nbank*nc, nif, ntime) = vcat. */
BLDP_API int bldp_stitch_f32(int nbank, const float *gathered, int64_t nc, int64_t nif, int64_t ntime,
                    float *out, void *stream);

/* In place on data (nchan, nif, ntime): for every coarse channel the DC bin
 * (0-based nfpc/2) takes the value of its left neighbour. nfpc >= 2. */
BLDP_API int bldp_despike_f32(float *data, int64_t nchan, int64_t nif, int64_t ntime, int64_t nfpc,
                     void *stream);

/* Excess kurtosis over time of every (channel, if) row of the window.
 * out is (nc, ni) float64 on the device. workspace: device scratch of
 * bldp_kurtosis_workspace_size() bytes, or NULL for a library-cached one. */
BLDP_API size_t bldp_kurtosis_workspace_size(int64_t nchan, int64_t nif, int64_t ntime, const int64_t *win);
/* Introspection (tests/bench): the kurtosis plan for this pointer and window.
 * info = {path (0 registers, 1 register tile, 2 streamed leaves + tree
 * merge, 3 two passes), K (level of the pairwise-sum blocks), leaf slots,
 * workspace bytes}.  Launches nothing. */
BLDP_API int bldp_kurtosis_plan_f32(const float *in, int64_t nchan, int64_t nif, int64_t ntime,
                                    const int64_t *win, int64_t info[4]);
BLDP_API int bldp_kurtosis_f32(const float *in, int64_t nchan, int64_t nif, int64_t ntime,
                      const int64_t *win, double *out, void *workspace, void *stream);

/* Kurtosis of every bank of a band resident on one device, one set of
 * launches for all banks (the GBT.getkurtosis fan-out, src/gbt.jl:81-88).
 * in[] is a HOST array of device pointers; out is nbank (nc, ni) float64
 * matrices back to back on the device. */
BLDP_API int bldp_band_kurtosis_f32(int nbank, const float *const *in, int64_t nchan,
                                    int64_t nif, int64_t ntime, const int64_t *win, double *out,
                                    void *stream);

/* Host-pointer form of bldp_kurtosis_f32 for a worker holding the data in
 * host memory: the window is staged on device `dev`, out (nc, ni) float64 is
 * host memory.  Synchronous. */
BLDP_API int bldp_kurtosis_host_f32(int dev, const float *in, int64_t nchan, int64_t nif,
                                    int64_t ntime, const int64_t *win, double *out);

/* Element types other than Float32 (what Blio maps SIGPROC nbits 8 / 16 to, and
 * what HDF5.jl returns for an integer or Float64 dataset: the reference's
 * readers hand any of them to fqav / kurtosis, src/gbtworkerfunctions.jl:173,
 * 181-188, 197-202). */
enum bldp_dtype {
  BLDP_DT_F32 = 0, BLDP_DT_F64 = 1, BLDP_DT_U8 = 2, BLDP_DT_U16 = 3, BLDP_DT_U32 = 4,
  BLDP_DT_U64 = 5, BLDP_DT_I8 = 6, BLDP_DT_I16 = 7, BLDP_DT_I32 = 8, BLDP_DT_I64 = 9
};
/* Element type of fqav's result for input `dtype` and `op`, Julia's:
 *   sum   UInt8/16/32/64 -> UInt64, Int8/16/32/64 -> Int64 (Base.add_sum
 *         widening; exact, wrapping on 64-bit overflow), Float32 / Float64 kept;
 *   mean  Float64 (Float32 kept);  max / min  the input type.
 * Returns the bldp_dtype, or BLDP_EINVAL. */
BLDP_API int bldp_reduce_out_dtype(int dtype, int op);
/* bldp_reduce_strided_f32 for any bldp_dtype: in holds `dtype` elements, out
 * bldp_reduce_out_dtype(dtype, op) elements (strides in elements).  Float32
 * input takes the Float32 kernels; the others one lane per output in the
 * reference's order (integer sums exact).  Device pointers, asynchronous. */
BLDP_API int bldp_reduce_strided(int dtype, const void *in, int64_t nchan, int64_t nif,
                                 int64_t ntime, const int64_t *win, int64_t fqavby, int64_t tavby,
                                 int op, void *out, int64_t out_ld_i, int64_t out_ld_t,
                                 void *stream);
/* getkurtosis for any bldp_dtype (StatsBase's recipe; Float64 arithmetic for
 * integer and Float64 rows: Base.sum's pairwise Float64 mean, sequential
 * moments; 8- and 16-bit rows from exact integer power sums, within 160 2^-53 of
 * the exactly rounded kurtosis and (3 nt + 175) 2^-53 relative of the
 * recipe on k + 3, plan option "typed_kurt").  out
 * (nc, ni) float64 on the device.  Asynchronous. */
BLDP_API int bldp_kurtosis(int dtype, const void *in, int64_t nchan, int64_t nif, int64_t ntime,
                           const int64_t *win, double *out, void *stream);
/* bldp_reduce_strided / bldp_kurtosis prepared once for fixed buffers (ABI 5;
 * any bldp_dtype, Float32 included): the checks, window and plan are taken
 * here, and each bldp_reduce_launch(handle, stream) only queues the kernel(s)
 * -- what a worker re-reducing the same per-file buffers pays per call
 * (src/gbtworkerfunctions.jl:171-177,191-195).  Same results and errors as
 * the unprepared calls; released with bldp_reduce_release.  Bound to the
 * current device.  bldp_reduce_launch_timed takes these handles too: the
 * Float32 reduce's own dispatches carry the events, the other kinds record
 * them on the stream around the launch. */
BLDP_API int bldp_reduce_prepare(int dtype, const void *in, int64_t nchan, int64_t nif,
                                 int64_t ntime, const int64_t *win, int64_t fqavby, int64_t tavby,
                                 int op, void *out, int64_t out_ld_i, int64_t out_ld_t,
                                 bldp_reduce_op_t *handle);
BLDP_API int bldp_kurtosis_prepare(int dtype, const void *in, int64_t nchan, int64_t nif,
                                   int64_t ntime, const int64_t *win, double *out,
                                   bldp_reduce_op_t *handle);
/* Host-memory forms (what a Julia worker holding the mmap'ed / read array
 * calls): the window's span is copied to device `dev`, reduced there, and the
 * result copied back into host `out` (dense (nco, ni, nto) of the output type;
 * (nc, ni) float64 for kurtosis).  Synchronous. */
BLDP_API int bldp_reduce_host(int dev, int dtype, const void *in, int64_t nchan, int64_t nif,
                              int64_t ntime, const int64_t *win, int64_t fqavby, int64_t tavby,
                              int op, void *out);
BLDP_API int bldp_kurtosis_host(int dev, int dtype, const void *in, int64_t nchan, int64_t nif,
                                int64_t ntime, const int64_t *win, double *out);

/* HDF5 filter 32008 (bitshuffle + LZ4) chunks, the codec of compressed
 * rawspec FBH5 products (H5Zbitshuffle, reference Project.toml:10; read at
 * src/gbtworkerfunctions.jl:181-187).  A chunk is the raw bytes H5Dread_chunk
 * returns: 12-byte header (uint64 BE uncompressed bytes, uint32 BE block
 * bytes), LZ4 blocks of bit-transposed elements, raw tail of n % 8 elements. */
BLDP_API int bldp_bslz4_info(const void *chunk, size_t nbytes, uint64_t *uncompressed_bytes,
                             uint32_t *block_bytes);
/* Decode one chunk on the host into out (exactly uncompressed_bytes). */
BLDP_API int bldp_bslz4_decode_host(const void *chunk, size_t nbytes, int elem_size, void *out,
                                    size_t out_bytes);
/* Decode nchunk chunks on the GPU.  comp_host and comp_dev hold the same
 * concatenated chunk bytes (the host copy is parsed into a block table, the
 * device copy is decoded); chunk k spans [chunk_off[k], +chunk_len[k]) and
 * decodes to out_dev + out_off[k] (bytes), a slot of out_len[k] bytes: a
 * chunk whose header claims any other size is rejected (BLDP_EINVAL) before
 * anything is launched, so no chunk writes outside its slot.  Synchronous:
 * returns after the decode finished, BLDP_EINVAL if any block is corrupt. */
BLDP_API int bldp_bslz4_decode_dev(int nchunk, const uint8_t *comp_host, const uint8_t *comp_dev,
                                   const uint64_t *chunk_off, const uint64_t *chunk_len,
                                   int elem_size, uint8_t *out_dev, const uint64_t *out_off,
                                   const uint64_t *out_len, void *stream);

/* Asynchronous form: queues the decode on `stream` and returns; error bits
 * are OR-ed into *err_dev (device int, zeroed by the caller before its first
 * call).  The host copy comp_host may be reused once the call returns.
 * bldp_bslz4_error synchronizes `stream` and turns *err_dev into a return
 * code (BLDP_EINVAL for a corrupt block). */
BLDP_API int bldp_bslz4_decode_dev_async(int nchunk, const uint8_t *comp_host,
                                         const uint8_t *comp_dev, const uint64_t *chunk_off,
                                         const uint64_t *chunk_len, int elem_size,
                                         uint8_t *out_dev, const uint64_t *out_off,
                                         const uint64_t *out_len, int *err_dev, void *stream);
BLDP_API int bldp_bslz4_error(const int *err_dev, void *stream);

/* The stored chunks of a chunked FBH5 window, file -> device, natively (the
 * chunk reads and filter 32008 of h5["data"][idxs...],
 * src/gbtworkerfunctions.jl:181-187).  Chunk k (stored_len[k] bytes at
 * file_off[k] of the open file `fd`; 0 bytes = never written) is read with
 * parallel preads (a persistent pool of reader threads per device: 16, or 4
 * fewer than the process's CPU quota when that is less, BLDP_READ_THREADS
 * overrides; they run on the CPUs of the GPU's NUMA node when the caller may
 * use at least half as many CPUs there, and the pinned slots are placed on
 * that node unless the calling thread has a memory policy of its own,
 * BLDP_READ_AFFINITY=0 / BLDP_SLOT_NUMA=0 undo that)
 * into host_pinned + stage_off[k] (both staging buffers hold stage_bytes;
 * dev_out holds out_bytes: every table entry is checked against them before
 * anything is read).  host_pinned NULL (since ABI 4): the reads are staged
 * through the device's library-owned pinned slot ring instead (the one
 * bldp_runs_to_device uses, 8 x 32 MiB; a batch whose staged range is larger
 * takes 2 slots of that size, released when the call returns), batch b in
 * slot b % nslot once that slot's previous copy is done, so pinned host memory
 * stays bounded whatever the window's size: 256 MiB between calls, at most
 * 2 x the largest batch during one; the call then also waits for its last
 * copy before returning.
 * Chunks [batch_end[b-1], batch_end[b]) form
 * batch b: once its reads land, its staged byte range is copied to dev_stage
 * (same offsets) on copy_stream, `stream` waits for that copy, and the batch's
 * chunks are decoded on `stream` into dev_out + k * out_chunk_bytes
 * (bitshuffle + LZ4, bldp_bslz4_decode_dev_async with err_dev; filter_mask
 * bit 0 set = stored without the filter: copied raw; dev_out may be NULL when
 * every chunk is raw: the staged bytes are the output).  Batch b + 1 is read
 * while batch b is copied and decoded.  Returns once every read has landed
 * and every copy and decode is queued; bldp_bslz4_error(err_dev, stream)
 * then synchronizes and reports corrupt blocks.  stats (NULL or 4 doubles):
 * ms to the first queued copy, ms to the last queued work, pread pieces,
 * reader threads. */
BLDP_API int bldp_chunks_to_device(int fd, int64_t nchunk, const int64_t *file_off,
                                   const int64_t *stored_len, const int64_t *stage_off,
                                   const uint32_t *filter_mask, int64_t nbatch,
                                   const int64_t *batch_end, void *host_pinned, void *dev_stage,
                                   int64_t stage_bytes, void *dev_out, int64_t out_chunk_bytes,
                                   int64_t out_bytes, int *err_dev, void *copy_stream,
                                   void *stream, double *stats);

/* bldp_chunks_to_device over the chunks of several files: chunk k is in the
 * open file fd[k] (the banks of a band of compressed FBH5 files read as one
 * stream of batches and decoded into one chunk grid per bank: GBT.getband,
 * src/gbt.jl:69-79,103; src/gbtworkerfunctions.jl:181-187).  Same staging,
 * batches, decode, streams, errors and return as bldp_chunks_to_device (ABI 4). */
BLDP_API int bldp_file_chunks_to_device(int64_t nchunk, const int *fd, const int64_t *file_off,
                                        const int64_t *stored_len, const int64_t *stage_off,
                                        const uint32_t *filter_mask, int64_t nbatch,
                                        const int64_t *batch_end, void *host_pinned,
                                        void *dev_stage, int64_t stage_bytes, void *dev_out,
                                        int64_t out_chunk_bytes, int64_t out_bytes, int *err_dev,
                                        void *copy_stream, void *stream, double *stats);

/* Raw byte runs of a file (an uncompressed contiguous FBH5 `data` dataset or
 * a SIGPROC data block: src/gbtworkerfunctions.jl:171-189) into a dense device
 * block: run r (len[r] bytes at file_off[r]) lands at dev_dst + the sum of
 * the earlier runs' lengths (dev_dst holds dst_bytes).  The block is cut
 * into batches of slot_bytes;
 * the reader threads pread batch b into library-owned pinned slot b % nslot
 * once that slot's previous copy is done, and each batch is copied to the
 * device on copy_stream as soon as its reads land.  Returns after every copy
 * is done; `stream` waits for the last.  stats as bldp_chunks_to_device. */
BLDP_API int bldp_runs_to_device(int fd, int64_t nrun, const int64_t *file_off,
                                 const int64_t *len, void *dev_dst, int64_t dst_bytes,
                                 int64_t slot_bytes, int nslot, void *copy_stream, void *stream,
                                 double *stats);

/* bldp_runs_to_device over runs of several files: run r is in the open file
 * fd[r] (the banks of a band read as one stream of batches into one device
 * block: GBT.getband, src/gbt.jl:69-79,103).  Same batching, slots, streams
 * and return as bldp_runs_to_device. */
BLDP_API int bldp_file_runs_to_device(int64_t nrun, const int *fd, const int64_t *file_off,
                                      const int64_t *len, void *dev_dst, int64_t dst_bytes,
                                      int64_t slot_bytes, int nslot, void *copy_stream,
                                      void *stream, double *stats);

/* Gather a window (Julia order, dense (nc, ni, nt) out) from decoded chunks:
 * packed holds the chunks of a chunk-aligned bounding box back to back in
 * chunk-grid order [gt][gi][gc], each chunk C-order [ct][ci][cc].
 * chunk = {ct, ci, cc}, box0 = {t, i, c} of the box's first element,
 * grid = {gt, gi, gc} chunks in the box, win = the usual 9-int window in
 * dataset coordinates (must lie inside the box). */
BLDP_API int bldp_unchunk_f32(const float *packed, const int64_t chunk[3], const int64_t box0[3],
                              const int64_t grid[3], const int64_t *win, float *out,
                              void *stream);

/* fqav(r::AbstractRange, n): first/step/length of the averaged axis. */
BLDP_API int bldp_fqav_range(double first, double step, int64_t len, int64_t n, double *out_first,
                    double *out_step, int64_t *out_len);

/* Synthetic BL-like filterbank (nchan, nif, ntime) on the device:
 * kind 0 = gamma(2, 5e8) x bandpass scallop x DC spike (nfpc bins per coarse
 * channel); kind 1 = integer-valued 0..255 (order-independent exact sums). */
BLDP_API int bldp_synth_f32(float *out, int64_t nchan, int64_t nif, int64_t ntime, int64_t nfpc,
                   uint64_t seed, int kind, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* BLDP_H */
