// runtime.hip — library-owned per-device state ("device staging
// buffers are library-owned and cached per device"):
//   * bldp_init / bldp_finalize;
//   * a pool of host-staging pipelines (two streams + device buffers) per
//     device, so the host-array entry points allocate nothing per call and
//     concurrent callers (GBT.getdata's per-worker fan-out, src/gbt.jl:75-77)
//     each get their own pipeline;
//   * one persistent worker stream per device for the multi-GPU band call;
//   * page-locking of long-lived caller host buffers.
#include <cstring>
#include <map>
#include <mutex>
#include <set>
#include <vector>

#include "bldp_impl.h"

namespace bldp {
namespace {

constexpr size_t kStageCacheCap = (size_t)1 << 30;  // larger buffers are per call

std::mutex g_mu;
std::map<int, std::vector<Stager *>> g_idle;  // idle pipelines per device
std::vector<Stager *> g_all;
std::map<int, hipStream_t> g_dev_stream;
std::set<int> g_checked;  // devices verified to be gfx950
int g_busy = 0;

struct DevSwitch {
  int prev = -1;
  explicit DevSwitch(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    (void)hipSetDevice(dev);
  }
  ~DevSwitch() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};

// g_mu held
int check_device_locked(int dev) {
  if (g_checked.count(dev)) return BLDP_OK;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || dev < 0 || dev >= n)
    return set_error(BLDP_EINVAL, "device %d not available (%d visible)", dev, n);
  hipDeviceProp_t pr;
  if (hipGetDeviceProperties(&pr, dev) != hipSuccess)
    return set_error(BLDP_EHIP, "hipGetDeviceProperties(%d) failed", dev);
  if (std::strncmp(pr.gcnArchName, "gfx950", 6) != 0)
    return set_error(BLDP_EINVAL, "device %d is %s; libbldp_hip is built for gfx950 only", dev,
                     pr.gcnArchName);
  g_checked.insert(dev);
  return BLDP_OK;
}

int grow(Stager *s, int slot, size_t need) {
  if (s->bytes[slot] >= need) return BLDP_OK;
  if (s->buf[slot]) {
    (void)hipStreamSynchronize(s->st[slot & 1]);
    (void)hipFree(s->buf[slot]);
    s->buf[slot] = nullptr;
    s->bytes[slot] = 0;
  }
  const size_t want = need > ((size_t)1 << 20) ? need : ((size_t)1 << 20);
  if (hipMalloc(&s->buf[slot], want) != hipSuccess) {
    s->buf[slot] = nullptr;
    return set_error(BLDP_ENOMEM, "device %d: staging allocation of %zu bytes failed", s->dev,
                     want);
  }
  s->bytes[slot] = want;
  return BLDP_OK;
}

void destroy(Stager *s) {
  for (int k = 0; k < 4; ++k)
    if (s->buf[k]) (void)hipFree(s->buf[k]);
  for (void *p : s->temp) (void)hipFree(p);
  for (int b = 0; b < 2; ++b)
    if (s->st[b]) (void)hipStreamDestroy(s->st[b]);
  delete s;
}

}  // namespace

int stager_acquire(int dev, Stager **out) {
  *out = nullptr;
  std::lock_guard<std::mutex> lk(g_mu);
  int rc = check_device_locked(dev);
  if (rc) return rc;
  auto &idle = g_idle[dev];
  if (!idle.empty()) {
    *out = idle.back();
    idle.pop_back();
    ++g_busy;
    return BLDP_OK;
  }
  DevSwitch sw(dev);
  Stager *s = new Stager();
  s->dev = dev;
  for (int b = 0; b < 2; ++b)
    if (hipStreamCreateWithFlags(&s->st[b], hipStreamNonBlocking) != hipSuccess) {
      destroy(s);
      return set_error(BLDP_EHIP, "device %d: stream creation failed", dev);
    }
  g_all.push_back(s);
  ++g_busy;
  *out = s;
  return BLDP_OK;
}

int stager_buffer(Stager *s, int slot, size_t need, void **p) {
  *p = nullptr;
  if (need > kStageCacheCap) {  // too big to keep: allocated for this call only
    void *t = nullptr;
    if (hipMalloc(&t, need) != hipSuccess)
      return set_error(BLDP_ENOMEM, "device %d: staging allocation of %zu bytes failed", s->dev,
                       need);
    s->temp.push_back(t);
    *p = t;
    return BLDP_OK;
  }
  int rc = grow(s, slot, need);
  if (rc) return rc;
  *p = s->buf[slot];
  return BLDP_OK;
}

void stager_release(Stager *s) {
  if (!s) return;
  if (!s->temp.empty()) {
    DevSwitch sw(s->dev);
    for (int b = 0; b < 2; ++b) (void)hipStreamSynchronize(s->st[b]);
    for (void *p : s->temp) (void)hipFree(p);
    s->temp.clear();
  }
  std::lock_guard<std::mutex> lk(g_mu);
  g_idle[s->dev].push_back(s);
  --g_busy;
}

int device_stream(int dev, hipStream_t *out) {
  std::lock_guard<std::mutex> lk(g_mu);
  int rc = check_device_locked(dev);
  if (rc) return rc;
  auto it = g_dev_stream.find(dev);
  if (it != g_dev_stream.end()) {
    *out = it->second;
    return BLDP_OK;
  }
  DevSwitch sw(dev);
  hipStream_t s = nullptr;
  if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess)
    return set_error(BLDP_EHIP, "device %d: stream creation failed", dev);
  g_dev_stream[dev] = s;
  *out = s;
  return BLDP_OK;
}

}  // namespace bldp

using namespace bldp;

extern "C" {

int bldp_init(int ndev, const int *devs) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return set_error(BLDP_EHIP, "hipGetDeviceCount failed");
  std::vector<int> list;
  if (devs) {
    if (ndev < 1) return set_error(BLDP_EINVAL, "ndev=%d with a device list", ndev);
    list.assign(devs, devs + ndev);
  } else {
    for (int d = 0; d < n; ++d) list.push_back(d);
  }
  for (int d : list) {
    hipStream_t s;
    int rc = device_stream(d, &s);  // validates the device (gfx950) and creates its stream
    if (rc) return rc;
    Stager *st = nullptr;
    rc = stager_acquire(d, &st);  // one warm host-staging pipeline per device
    if (rc) return rc;
    stager_release(st);
  }
  // Peer access between the listed devices: lets bldp_band_reduce_multi_f32's
  // kernels write the root's stitched product directly over xGMI.
  for (int d : list) {
    DevSwitch sw(d);
    for (int e : list) {
      if (e == d) continue;
      int can = 0;
      if (hipDeviceCanAccessPeer(&can, d, e) == hipSuccess && can) {
        (void)hipDeviceEnablePeerAccess(e, 0);  // already-enabled is fine
        (void)hipGetLastError();
      }
    }
  }
  return BLDP_OK;
}

int bldp_finalize(void) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (g_busy) return set_error(BLDP_EINVAL, "bldp_finalize: %d host pipelines still in use", g_busy);
  std::set<int> devs;
  for (Stager *s : g_all) devs.insert(s->dev);
  for (auto &kv : g_dev_stream) devs.insert(kv.first);
  for (int d : scratch_devices()) devs.insert(d);
  int prev = -1;
  (void)hipGetDevice(&prev);
  for (int d : devs) {  // drain everything that may still use library memory
    (void)hipSetDevice(d);
    (void)hipDeviceSynchronize();
  }
  for (Stager *s : g_all) {
    (void)hipSetDevice(s->dev);
    destroy(s);
  }
  g_all.clear();
  g_idle.clear();
  for (auto &kv : g_dev_stream) {
    (void)hipSetDevice(kv.first);
    (void)hipStreamDestroy(kv.second);
  }
  g_dev_stream.clear();
  scratch_release_all();
  fileio_release();  // the file readers' pinned slots and threads
  if (prev >= 0) (void)hipSetDevice(prev);
  return BLDP_OK;
}

int bldp_host_register(void *ptr, size_t bytes) {
  if (!ptr || bytes == 0) return set_error(BLDP_EINVAL, "null or empty host buffer");
  const hipError_t e = hipHostRegister(ptr, bytes, hipHostRegisterDefault);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    return set_error(BLDP_EHIP, "hipHostRegister(%zu bytes): %s", bytes, hipGetErrorString(e));
  }
  return BLDP_OK;
}

int bldp_host_unregister(void *ptr) {
  if (!ptr) return set_error(BLDP_EINVAL, "null host buffer");
  const hipError_t e = hipHostUnregister(ptr);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    return set_error(BLDP_EHIP, "hipHostUnregister: %s", hipGetErrorString(e));
  }
  return BLDP_OK;
}

}  // extern "C"
