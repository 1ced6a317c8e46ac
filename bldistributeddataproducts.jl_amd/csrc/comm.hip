// comm.hip — the band stitch across GPUs through the C ABI: RCCL over xGMI
// for hosts that run one process per GPU without torch (the Julia reference's
// Distributed.jl workers, one per bank: src/gbt.jl:75-77).
//
//   rank 0:        bldp_comm_id(id)                 -> send id to every rank
//   every rank:    bldp_comm_init(dev, nranks, rank, id, &comm)
//                  bldp_band_reduce_f32(... its banks ..., slice, stream)
//                  bldp_band_gather_f32(comm, root, slice, count, gathered, stream)
//   root:          bldp_stitch_f32(nranks, gathered, ...) when ni*nto > 1
//   every rank:    bldp_comm_destroy(comm)
//
// This is the ncclGather of SURVEY §8e (rccl.h:745): each rank's reduced
// slice (its banks in vcat order, dense (nco_local, ni, nto)) lands
// rank-major on the root.  RCCL is loaded with dlopen on first use, so
// libbldp_hip links nothing beyond the HIP runtime and the single-GPU entry
// points work where RCCL is absent.
#include <dlfcn.h>
#include <rccl/rccl.h>

#include <cstring>
#include <mutex>

#include "bldp_impl.h"

namespace {

struct Rccl {
  bool tried = false;
  void *h = nullptr;
  ncclResult_t (*get_unique_id)(ncclUniqueId *) = nullptr;
  ncclResult_t (*comm_init_rank)(ncclComm_t *, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
  ncclResult_t (*gather)(const void *, void *, size_t, ncclDataType_t, int, ncclComm_t,
                         hipStream_t) = nullptr;
  const char *(*error_string)(ncclResult_t) = nullptr;
};

std::mutex g_rccl_mu;
Rccl g_rccl;

// Resolve librccl once; BLDP_EINVAL with the dlerror text when absent.
int rccl(Rccl **out) {
  std::lock_guard<std::mutex> lk(g_rccl_mu);
  if (!g_rccl.tried) {
    g_rccl.tried = true;
    const char *names[] = {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"};
    for (const char *n : names)
      if ((g_rccl.h = dlopen(n, RTLD_NOW | RTLD_GLOBAL))) break;
    if (g_rccl.h) {
      g_rccl.get_unique_id = (decltype(g_rccl.get_unique_id))dlsym(g_rccl.h, "ncclGetUniqueId");
      g_rccl.comm_init_rank = (decltype(g_rccl.comm_init_rank))dlsym(g_rccl.h, "ncclCommInitRank");
      g_rccl.comm_destroy = (decltype(g_rccl.comm_destroy))dlsym(g_rccl.h, "ncclCommDestroy");
      g_rccl.gather = (decltype(g_rccl.gather))dlsym(g_rccl.h, "ncclGather");
      g_rccl.error_string = (decltype(g_rccl.error_string))dlsym(g_rccl.h, "ncclGetErrorString");
    }
  }
  if (!g_rccl.get_unique_id || !g_rccl.comm_init_rank || !g_rccl.comm_destroy ||
      !g_rccl.gather || !g_rccl.error_string)
    return bldp::set_error(BLDP_EINVAL, "RCCL (librccl.so.1 with ncclGather) not available: %s",
                           g_rccl.h ? "missing symbols" : dlerror());
  *out = &g_rccl;
  return BLDP_OK;
}

// A communicator bound to its device (every call switches to it).
struct Comm {
  ncclComm_t nccl = nullptr;
  int dev = -1, nranks = 0, rank = -1;
};

struct DevGuard {
  int prev = -1;
  explicit DevGuard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    (void)hipSetDevice(dev);
  }
  ~DevGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};

int nccl_fail(Rccl *r, ncclResult_t e, const char *what) {
  return bldp::set_error(BLDP_ECOMM, "%s: %s", what, r->error_string(e));
}

}  // namespace

extern "C" {

int bldp_comm_id(uint8_t id[BLDP_COMM_ID_BYTES]) {
  if (!id) return bldp::set_error(BLDP_EINVAL, "null id buffer");
  Rccl *r;
  int rc = rccl(&r);
  if (rc) return rc;
  ncclUniqueId u;
  const ncclResult_t e = r->get_unique_id(&u);
  if (e != ncclSuccess) return nccl_fail(r, e, "ncclGetUniqueId");
  static_assert(sizeof(u) == BLDP_COMM_ID_BYTES, "ncclUniqueId size");
  std::memcpy(id, &u, sizeof u);
  return BLDP_OK;
}

int bldp_comm_init(int dev, int nranks, int rank, const uint8_t id[BLDP_COMM_ID_BYTES],
                   void **comm) {
  if (!comm || !id) return bldp::set_error(BLDP_EINVAL, "null comm or id pointer");
  *comm = nullptr;
  if (nranks < 1 || rank < 0 || rank >= nranks)
    return bldp::set_error(BLDP_EINVAL, "rank %d outside 0..%d", rank, nranks - 1);
  hipStream_t s;
  int rc = bldp::device_stream(dev, &s);  // validates dev (gfx950)
  if (rc) return rc;
  Rccl *r;
  rc = rccl(&r);
  if (rc) return rc;
  ncclUniqueId u;
  std::memcpy(&u, id, sizeof u);
  Comm *c = new Comm();
  c->dev = dev;
  c->nranks = nranks;
  c->rank = rank;
  DevGuard g(dev);
  const ncclResult_t e = r->comm_init_rank(&c->nccl, nranks, u, rank);  // collective
  if (e != ncclSuccess) {
    delete c;
    return nccl_fail(r, e, "ncclCommInitRank");
  }
  *comm = c;
  return BLDP_OK;
}

int bldp_comm_destroy(void *comm) {
  if (!comm) return BLDP_OK;
  Comm *c = static_cast<Comm *>(comm);
  Rccl *r;
  int rc = rccl(&r);
  if (rc) return rc;
  DevGuard g(c->dev);
  const ncclResult_t e = r->comm_destroy(c->nccl);
  delete c;
  if (e != ncclSuccess) return nccl_fail(r, e, "ncclCommDestroy");
  return BLDP_OK;
}

int bldp_band_gather_f32(void *comm, int root, const float *slice, int64_t count,
                         float *gathered, void *stream) {
  if (!comm) return bldp::set_error(BLDP_EINVAL, "null communicator");
  Comm *c = static_cast<Comm *>(comm);
  if (root < 0 || root >= c->nranks)
    return bldp::set_error(BLDP_EINVAL, "root %d outside 0..%d", root, c->nranks - 1);
  if (count < 0) return bldp::set_error(BLDP_EINVAL, "negative count");
  if (count == 0) return BLDP_OK;
  if (!slice) return bldp::set_error(BLDP_EINVAL, "null slice pointer");
  if (c->rank == root && !gathered)
    return bldp::set_error(BLDP_EINVAL, "null gathered pointer on the root");
  Rccl *r;
  int rc = rccl(&r);
  if (rc) return rc;
  DevGuard g(c->dev);
  const ncclResult_t e = r->gather(slice, gathered, (size_t)count, ncclFloat32, root, c->nccl,
                                   (hipStream_t)stream);
  if (e != ncclSuccess) return nccl_fail(r, e, "ncclGather");
  return BLDP_OK;
}

}  // extern "C"
