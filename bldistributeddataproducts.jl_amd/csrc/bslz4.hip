// bslz4.hip — HDF5 filter 32008 (bitshuffle + LZ4) chunk decoding, on the
// host and on the GPU.  This is the codec of compressed rawspec FBH5 products;
// the reference gets it from H5Zbitshuffle (Project.toml:10,
// src/gbtworkerfunctions.jl:3) during h5["data"][idxs...] (:181-187).
//
// Chunk layout (bitshuffle's HDF5 filter, LZ4 mode):
//   uint64 BE  uncompressed bytes  (n * elem_size)
//   uint32 BE  block size in bytes (block * elem_size)
//   n / block full blocks, then one block of (n % block) rounded down to a
//   multiple of 8 elements; each block = uint32 BE compressed size + an LZ4
//   block holding the bit-transposed elements (bit plane r = byte r/8, bit r%8
//   of every element, packed LSB-first);
//   then the last n % 8 elements, raw.
//
// GPU design: the host reads only each chunk's 12-byte header; a planner
// kernel (one thread per chunk) walks the block-size fields, already on the
// device, into a task table; then one wave per block stages the compressed bytes in LDS, decodes LZ4 into
// LDS (sequence parsing is wave-uniform, literal and match copies are spread
// over the 64 lanes, overlapping matches in rounds of `offset` bytes), then
// inverts the bit transpose with an 8x8 bit-matrix transpose per 8 elements
// straight into global memory.  Every read and write is bounds checked: a
// corrupt chunk sets an error word instead of touching memory out of range.
#include <algorithm>
#include <cstring>
#include <vector>

#include "bldp_impl.h"

namespace {

inline uint32_t be32(const uint8_t *p) {
  return (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3];
}
inline uint64_t be64(const uint8_t *p) { return (uint64_t)be32(p) << 32 | be32(p + 4); }

// 8x8 bit-matrix transpose: bit (row r, col c) at 8r+c moves to 8c+r.
__host__ __device__ inline uint64_t transpose8(uint64_t x) {
  uint64_t t;
  t = (x ^ (x >> 7)) & 0x00AA00AA00AA00AAull;
  x = x ^ t ^ (t << 7);
  t = (x ^ (x >> 14)) & 0x0000CCCC0000CCCCull;
  x = x ^ t ^ (t << 14);
  t = (x ^ (x >> 28)) & 0x00000000F0F0F0F0ull;
  x = x ^ t ^ (t << 28);
  return x;
}

// LZ4 block decode with full bounds checks.  Returns bytes written or -1.
int64_t lz4_block_host(const uint8_t *src, size_t slen, uint8_t *dst, size_t dcap) {
  size_t ip = 0, op = 0;
  while (ip < slen) {
    const uint8_t token = src[ip++];
    size_t lit = token >> 4;
    if (lit == 15) {
      uint8_t b;
      do {
        if (ip >= slen) return -1;
        b = src[ip++];
        lit += b;
      } while (b == 255);
    }
    if (ip + lit > slen || op + lit > dcap) return -1;
    memcpy(dst + op, src + ip, lit);
    ip += lit;
    op += lit;
    if (ip >= slen) break;  // the last sequence carries literals only
    if (ip + 2 > slen) return -1;
    const size_t off = (size_t)src[ip] | (size_t)src[ip + 1] << 8;
    ip += 2;
    size_t ml = token & 15;
    if (ml == 15) {
      uint8_t b;
      do {
        if (ip >= slen) return -1;
        b = src[ip++];
        ml += b;
      } while (b == 255);
    }
    ml += 4;
    if (off == 0 || off > op || op + ml > dcap) return -1;
    for (size_t i = 0; i < ml; ++i) dst[op + i] = dst[op - off + i];  // may overlap
    op += ml;
  }
  return (int64_t)op;
}

// planes: n elements (n % 8 == 0) of es bytes, bit plane r at r*(n/8).
void bitunshuffle_host(const uint8_t *planes, uint8_t *out, size_t n, size_t es) {
  const size_t rowb = n / 8;
  for (size_t g = 0; g < rowb; ++g)
    for (size_t j = 0; j < es; ++j) {
      uint64_t x = 0;
      for (int k = 0; k < 8; ++k) x |= (uint64_t)planes[(j * 8 + k) * rowb + g] << (8 * k);
      x = transpose8(x);
      for (int t = 0; t < 8; ++t) out[(8 * g + t) * es + j] = (uint8_t)(x >> (8 * t));
    }
}

struct Task {        // one unit of GPU work
  uint64_t src;      // byte offset of the LZ4 block (raw bytes when clen == RAW)
  uint64_t dst;      // byte offset in the output
  uint32_t clen;     // compressed bytes, or RAW
  uint32_t nelem;    // elements decoded by this task
};
constexpr uint32_t RAW = 0xFFFFFFFFu;

// Per-chunk geometry from its 12-byte header (host side, one read per chunk).
struct ChunkDesc {
  uint64_t src, len, dst;      // chunk bytes [src, src+len) -> output bytes at dst
  uint64_t n, block;           // elements, elements per full block
  uint32_t nfull, last, tail;  // full blocks, last partial block, raw tail elements
  uint32_t task0;              // first task index of this chunk
};

int describe_chunk(const uint8_t *c, uint64_t len, uint64_t src, uint64_t dst, int es,
                   ChunkDesc *d) {
  if (len < 12) return bldp::set_error(BLDP_EINVAL, "bslz4: chunk shorter than its header");
  const uint64_t nb = be64(c);
  const uint32_t bb = be32(c + 8);
  if (nb % es || bb % es || bb == 0 || (bb / es) % 8 || bb > (1u << 24))
    return bldp::set_error(BLDP_EINVAL, "bslz4: bad header (bytes %llu, block %u, elem %d)",
                           (unsigned long long)nb, bb, es);
  d->src = src;
  d->len = len;
  d->dst = dst;
  d->n = nb / es;
  d->block = bb / es;
  d->nfull = (uint32_t)(d->n / d->block);
  uint64_t last = d->n % d->block;
  d->last = (uint32_t)(last - last % 8);
  d->tail = (uint32_t)(d->n - (uint64_t)d->nfull * d->block - d->last);
  return BLDP_OK;
}

inline uint32_t ntasks(const ChunkDesc &d) {
  return d.nfull + (d.last ? 1 : 0) + (d.tail ? 1 : 0);
}

// LZ4 worst case for one block (LZ4_COMPRESSBOUND)
__host__ __device__ inline uint32_t lz4_bound(uint32_t n) { return n + n / 255 + 16; }

__device__ inline uint32_t be32_dev(const uint8_t *p) {
  return (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3];
}

// One thread per chunk walks its block-size fields (already on the device)
// into the task table; a block that overruns its chunk sets *err.
__global__ __launch_bounds__(64) void k_bslz4_plan(const uint8_t *__restrict__ comp,
                                                   const ChunkDesc *__restrict__ chunks,
                                                   int nchunk, int es, uint32_t cap,
                                                   Task *__restrict__ tasks, int *err) {
  const int k = blockIdx.x * 64 + threadIdx.x;
  if (k >= nchunk) return;
  const ChunkDesc d = chunks[k];
  uint64_t pos = d.src + 12, e = 0;
  const uint64_t end = d.src + d.len;
  const uint32_t nblk = d.nfull + (d.last ? 1 : 0);
  for (uint32_t b = 0; b < nblk; ++b) {
    const uint32_t ne = b < d.nfull ? (uint32_t)d.block : d.last;
    if (pos + 4 > end) { atomicOr(err, 2); return; }
    const uint32_t cl = be32_dev(comp + pos);
    if (cl > cap || pos + 4 + cl > end) { atomicOr(err, 2); return; }
    tasks[d.task0 + b] = Task{pos + 4, d.dst + e * es, cl, ne};
    pos += 4 + cl;
    e += ne;
  }
  if (pos + (uint64_t)d.tail * es != end) { atomicOr(err, 4); return; }
  if (d.tail) tasks[d.task0 + nblk] = Task{pos, d.dst + e * es, RAW, d.tail};
}

// Walk one chunk's headers into tasks; returns 0 or an error code.
int plan_chunk(const uint8_t *c, uint64_t len, uint64_t src0, uint64_t dst0, int es,
               std::vector<Task> &tasks, uint64_t *out_bytes, uint32_t *max_block) {
  if (len < 12) return bldp::set_error(BLDP_EINVAL, "bslz4: chunk shorter than its header");
  const uint64_t nb = be64(c);
  const uint32_t bb = be32(c + 8);
  if (nb % es || bb % es || bb == 0 || (bb / es) % 8)
    return bldp::set_error(BLDP_EINVAL, "bslz4: bad header (bytes %llu, block %u, elem %d)",
                           (unsigned long long)nb, bb, es);
  const uint64_t n = nb / es, block = bb / es;
  uint64_t pos = 12, e = 0;
  const uint64_t nfull = n / block;
  uint64_t last = n % block;
  last -= last % 8;
  for (uint64_t k = 0; k < nfull + (last ? 1 : 0); ++k) {
    const uint64_t ne = k < nfull ? block : last;
    if (pos + 4 > len) return bldp::set_error(BLDP_EINVAL, "bslz4: truncated block header");
    const uint32_t cl = be32(c + pos);
    if (cl == RAW || pos + 4 + cl > len)
      return bldp::set_error(BLDP_EINVAL, "bslz4: block %llu overruns the chunk",
                             (unsigned long long)k);
    tasks.push_back(Task{src0 + pos + 4, dst0 + e * es, cl, (uint32_t)ne});
    *max_block = std::max<uint32_t>(*max_block, std::max<uint32_t>(cl, (uint32_t)(ne * es)));
    pos += 4 + cl;
    e += ne;
  }
  const uint64_t tail = n - e;  // < 8 raw elements
  if (pos + tail * es != len)
    return bldp::set_error(BLDP_EINVAL, "bslz4: %llu trailing bytes, expected %llu",
                           (unsigned long long)(len - pos), (unsigned long long)(tail * es));
  if (tail) tasks.push_back(Task{src0 + pos, dst0 + e * es, RAW, (uint32_t)tail});
  *out_bytes = nb;
  return BLDP_OK;
}

// One wave per task.  Dynamic LDS: [0, cap) compressed bytes, [cap, 2cap) decoded.
__global__ __launch_bounds__(64) void k_bslz4(const uint8_t *__restrict__ comp,
                                              const Task *__restrict__ tasks, int ntask,
                                              uint8_t *__restrict__ out, int es, uint32_t cap,
                                              int *err) {
  extern __shared__ uint8_t lds[];
  const int lane = threadIdx.x;
  if (*err & 6) return;  // the planner rejected a chunk: the task table is incomplete
  const Task t = tasks[blockIdx.x];
  if (t.clen == RAW) {  // raw tail bytes of a chunk
    for (uint32_t i = lane; i < t.nelem * (uint32_t)es; i += 64) out[t.dst + i] = comp[t.src + i];
    return;
  }
  uint8_t *in = lds, *dec = lds + cap;
  const uint32_t clen = t.clen, nbytes = t.nelem * (uint32_t)es;
  if (clen > cap) {
    if (lane == 0) atomicOr(err, 1);
    return;
  }
  for (uint32_t i = lane; i < clen; i += 64) in[i] = comp[t.src + i];
  __syncthreads();
  // LZ4: every lane parses the same sequence (wave-uniform control flow)
  uint32_t ip = 0, op = 0;
  bool bad = false;
  while (ip < clen) {
    const uint32_t token = in[ip++];
    uint32_t lit = token >> 4;
    if (lit == 15) {
      uint32_t b;
      do {
        if (ip >= clen) { bad = true; break; }
        b = in[ip++];
        lit += b;
      } while (b == 255);
      if (bad) break;
    }
    if (ip + lit > clen || op + lit > nbytes) { bad = true; break; }
    for (uint32_t i = lane; i < lit; i += 64) dec[op + i] = in[ip + i];
    ip += lit;
    op += lit;
    if (ip >= clen) break;
    if (ip + 2 > clen) { bad = true; break; }
    const uint32_t off = (uint32_t)in[ip] | (uint32_t)in[ip + 1] << 8;
    ip += 2;
    uint32_t ml = token & 15;
    if (ml == 15) {
      uint32_t b;
      do {
        if (ip >= clen) { bad = true; break; }
        b = in[ip++];
        ml += b;
      } while (b == 255);
      if (bad) break;
    }
    ml += 4;
    if (off == 0 || off > op || op + ml > nbytes) { bad = true; break; }
    __syncthreads();  // literals of this sequence are visible to the match copy
    // dst[op + i] = dst[op - off + i]; with off < ml the source overlaps the
    // destination, so copy in rounds of at most `off` bytes
    const uint32_t step = off < 64 ? off : 64;
    for (uint32_t r = 0; r < ml; r += step) {
      const uint32_t i = r + lane;
      if (lane < step && i < ml) dec[op + i] = dec[op - off + i];
      __syncthreads();
    }
    op += ml;
  }
  if (bad || op != nbytes) {
    if (lane == 0) atomicOr(err, 1);
    return;
  }
  __syncthreads();
  // inverse bit transpose: lane owns groups of 8 elements
  const uint32_t rowb = t.nelem / 8;
  if (es == 4) {
    for (uint32_t g = lane; g < rowb; g += 64) {
      uint32_t w[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        uint64_t x = 0;
#pragma unroll
        for (int k = 0; k < 8; ++k) x |= (uint64_t)dec[(j * 8 + k) * rowb + g] << (8 * k);
        x = transpose8(x);
#pragma unroll
        for (int q = 0; q < 8; ++q) w[q] |= (uint32_t)((x >> (8 * q)) & 0xFF) << (8 * j);
      }
      uint32_t *o = reinterpret_cast<uint32_t *>(out + t.dst) + 8 * g;
#pragma unroll
      for (int q = 0; q < 8; ++q) o[q] = w[q];
    }
  } else {
    for (uint32_t g = lane; g < rowb; g += 64)
      for (int j = 0; j < es; ++j) {
        uint64_t x = 0;
        for (int k = 0; k < 8; ++k) x |= (uint64_t)dec[(j * 8 + k) * rowb + g] << (8 * k);
        x = transpose8(x);
        for (int q = 0; q < 8; ++q) out[t.dst + (8 * g + q) * es + j] = (uint8_t)(x >> (8 * q));
      }
  }
}

}  // namespace

extern "C" {

BLDP_API int bldp_bslz4_info(const void *chunk, size_t nbytes, uint64_t *uncompressed_bytes,
                             uint32_t *block_bytes) {
  if (!chunk || nbytes < 12 || !uncompressed_bytes || !block_bytes)
    return bldp::set_error(BLDP_EINVAL, "bslz4: null pointer or short chunk");
  *uncompressed_bytes = be64((const uint8_t *)chunk);
  *block_bytes = be32((const uint8_t *)chunk + 8);
  return BLDP_OK;
}

BLDP_API int bldp_bslz4_decode_host(const void *chunk, size_t nbytes, int elem_size, void *out,
                                    size_t out_bytes) {
  if (!chunk || (!out && out_bytes) || elem_size <= 0)
    return bldp::set_error(BLDP_EINVAL, "bslz4: bad argument");
  std::vector<Task> tasks;
  uint64_t total = 0;
  uint32_t maxb = 0;
  int rc = plan_chunk((const uint8_t *)chunk, nbytes, 0, 0, elem_size, tasks, &total, &maxb);
  if (rc) return rc;
  if (total != out_bytes)
    return bldp::set_error(BLDP_EINVAL, "bslz4: chunk holds %llu bytes, output has %zu",
                           (unsigned long long)total, out_bytes);
  const uint8_t *c = (const uint8_t *)chunk;
  uint8_t *o = (uint8_t *)out;
  std::vector<uint8_t> dec(maxb);
  for (const Task &t : tasks) {
    const size_t nb = (size_t)t.nelem * elem_size;
    if (t.clen == RAW) {
      memcpy(o + t.dst, c + t.src, nb);
      continue;
    }
    if (lz4_block_host(c + t.src, t.clen, dec.data(), nb) != (int64_t)nb)
      return bldp::set_error(BLDP_EINVAL, "bslz4: corrupt LZ4 block at byte %llu",
                             (unsigned long long)t.src);
    bitunshuffle_host(dec.data(), o + t.dst, t.nelem, elem_size);
  }
  return BLDP_OK;
}

// Shared by the synchronous and asynchronous entry points: describe the
// chunks on the host, then queue the planner and the decoder on `s`; error
// bits are OR-ed into *derr (device memory).
// The host copy of chunk k's header is at comp_host + (chunk_off[k] - host_base)
// (host_base 0: the host and device staging buffers share offsets; the chunk
// reader's slot ring passes the batch's first staged offset).
static int decode_launch(int nchunk, const uint8_t *comp_host, const uint8_t *comp_dev,
                         const uint64_t *chunk_off, const uint64_t *chunk_len, int elem_size,
                         uint8_t *out_dev, const uint64_t *out_off, const uint64_t *out_len,
                         int *derr_user, hipStream_t s, int **derr_used,
                         bldp::ScratchLease &lease, uint64_t host_base = 0) {
  if (nchunk < 0 || (nchunk && (!comp_host || !comp_dev || !chunk_off || !chunk_len ||
                                !out_dev || !out_off || !out_len)) ||
      elem_size <= 0 || elem_size > 64)
    return bldp::set_error(BLDP_EINVAL, "bslz4: bad argument");
  if (elem_size == 4 && ((uintptr_t)out_dev & 3))
    return bldp::set_error(BLDP_EINVAL, "bslz4: output must be 4-byte aligned");
  // host: one 12-byte header per chunk -> geometry and task ranges
  std::vector<ChunkDesc> descs(nchunk);
  uint64_t ntask = 0;
  uint32_t maxbb = 0;
  for (int k = 0; k < nchunk; ++k) {
    if (chunk_off[k] < host_base)
      return bldp::set_error(BLDP_EINVAL, "bslz4: chunk %d below the host staging base", k);
    int rc = describe_chunk(comp_host + (chunk_off[k] - host_base), chunk_len[k], chunk_off[k],
                            out_off[k],
                            elem_size, &descs[k]);
    if (rc) return rc;
    // the header's byte count decides how much the kernels write: it must be
    // the caller's slot exactly (a corrupt or foreign chunk never spills over)
    if (descs[k].n * (uint64_t)elem_size != out_len[k])
      return bldp::set_error(BLDP_EINVAL,
                             "bslz4: chunk %d decodes to %llu bytes, its output slot holds %llu",
                             k, (unsigned long long)(descs[k].n * elem_size),
                             (unsigned long long)out_len[k]);
    if (elem_size == 4 && (out_off[k] & 3))
      return bldp::set_error(BLDP_EINVAL, "bslz4: output offsets must be 4-byte aligned");
    descs[k].task0 = (uint32_t)ntask;
    ntask += ntasks(descs[k]);
    if (ntask > INT32_MAX) return bldp::set_error(BLDP_EINVAL, "bslz4: too many blocks");
    maxbb = std::max<uint32_t>(maxbb, (uint32_t)(descs[k].block * elem_size));
  }
  *derr_used = nullptr;
  if (ntask == 0) return BLDP_OK;
  const uint32_t cap = (lz4_bound(maxbb) + 15) & ~15u;
  if ((size_t)cap + (((size_t)maxbb + 15) & ~(size_t)15) > 64 * 1024)
    return bldp::set_error(BLDP_EINVAL, "bslz4: block of %u bytes exceeds the LDS plan", maxbb);
  const size_t dbytes = ((descs.size() * sizeof(ChunkDesc)) + 255) & ~(size_t)255;
  const size_t tbytes = ((ntask * sizeof(Task)) + 255) & ~(size_t)255;
  // the caller holds the lease until it no longer reads the scratch
  int rc = bldp::scratch_lease(s, dbytes + tbytes + 256, &lease);
  if (rc) return rc;
  void *ws = lease.ptr;
  ChunkDesc *ddesc = (ChunkDesc *)ws;
  Task *dtask = (Task *)((char *)ws + dbytes);
  int *derr = derr_user ? derr_user : (int *)((char *)ws + dbytes + tbytes);
  if (hipMemcpyAsync(ddesc, descs.data(), descs.size() * sizeof(ChunkDesc),
                     hipMemcpyHostToDevice, s) != hipSuccess ||
      (!derr_user && hipMemsetAsync(derr, 0, sizeof(int), s) != hipSuccess))
    return bldp::set_error(BLDP_EHIP, "bslz4: descriptor upload failed");
  hipLaunchKernelGGL(k_bslz4_plan, dim3((unsigned)((nchunk + 63) / 64)), dim3(64), 0, s,
                     comp_dev, ddesc, nchunk, elem_size, cap, dtask, derr);
  const uint32_t dcap = (maxbb + 15) & ~15u;
  hipLaunchKernelGGL(k_bslz4, dim3((unsigned)ntask), dim3(64), cap + dcap, s, comp_dev, dtask,
                     (int)ntask, out_dev, elem_size, cap, derr);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return bldp::set_error(BLDP_EHIP, "bslz4 launch: %s", hipGetErrorString(e));
  *derr_used = derr;
  return BLDP_OK;
}

static int decode_error(int herr) {
  if (herr & 6) return bldp::set_error(BLDP_EINVAL, "bslz4: block table overruns a chunk");
  if (herr) return bldp::set_error(BLDP_EINVAL, "bslz4: corrupt LZ4 block on the device");
  return BLDP_OK;
}

BLDP_API int bldp_bslz4_decode_dev(int nchunk, const uint8_t *comp_host, const uint8_t *comp_dev,
                                   const uint64_t *chunk_off, const uint64_t *chunk_len,
                                   int elem_size, uint8_t *out_dev, const uint64_t *out_off,
                                   const uint64_t *out_len, void *stream) {
  hipStream_t s = (hipStream_t)stream;
  int *derr = nullptr;
  bldp::ScratchLease lease;  // held through the error read-back (derr lives in scratch)
  int rc = decode_launch(nchunk, comp_host, comp_dev, chunk_off, chunk_len, elem_size, out_dev,
                         out_off, out_len, nullptr, s, &derr, lease);
  if (rc || !derr) return rc;
  int herr = 0;
  if (hipMemcpyAsync(&herr, derr, sizeof(int), hipMemcpyDeviceToHost, s) != hipSuccess ||
      hipStreamSynchronize(s) != hipSuccess)
    return bldp::set_error(BLDP_EHIP, "bslz4: synchronize failed");
  return decode_error(herr);
}

BLDP_API int bldp_bslz4_decode_dev_async(int nchunk, const uint8_t *comp_host,
                                         const uint8_t *comp_dev, const uint64_t *chunk_off,
                                         const uint64_t *chunk_len, int elem_size,
                                         uint8_t *out_dev, const uint64_t *out_off,
                                         const uint64_t *out_len, int *err_dev, void *stream) {
  if (!err_dev) return bldp::set_error(BLDP_EINVAL, "bslz4: null error word");
  int *derr = nullptr;
  bldp::ScratchLease lease;  // until the planner and decoder are queued
  return decode_launch(nchunk, comp_host, comp_dev, chunk_off, chunk_len, elem_size, out_dev,
                       out_off, out_len, err_dev, (hipStream_t)stream, &derr, lease);
}

BLDP_API int bldp_bslz4_error(const int *err_dev, void *stream) {
  if (!err_dev) return bldp::set_error(BLDP_EINVAL, "bslz4: null error word");
  int herr = 0;
  hipStream_t s = (hipStream_t)stream;
  if (hipMemcpyAsync(&herr, err_dev, sizeof(int), hipMemcpyDeviceToHost, s) != hipSuccess ||
      hipStreamSynchronize(s) != hipSuccess)
    return bldp::set_error(BLDP_EHIP, "bslz4: synchronize failed");
  return decode_error(herr);
}

}  // extern "C"

// bldp_bslz4_decode_dev_async with the host headers at comp_host +
// (chunk_off[k] - host_base): the chunk reader's slot ring (fileio.hip).
int bldp::bslz4_decode_async_at(int nchunk, const uint8_t *comp_host, uint64_t host_base,
                                const uint8_t *comp_dev, const uint64_t *chunk_off,
                                const uint64_t *chunk_len, int elem_size, uint8_t *out_dev,
                                const uint64_t *out_off, const uint64_t *out_len, int *err_dev,
                                hipStream_t s) {
  if (!err_dev) return bldp::set_error(BLDP_EINVAL, "bslz4: null error word");
  int *derr = nullptr;
  bldp::ScratchLease lease;  // until the planner and decoder are queued
  return decode_launch(nchunk, comp_host, comp_dev, chunk_off, chunk_len, elem_size, out_dev,
                       out_off, out_len, err_dev, s, &derr, lease, host_base);
}
