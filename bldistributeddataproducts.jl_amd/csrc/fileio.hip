// fileio.hip — native file readers: the stored chunks of a chunked FBH5
// window (or the byte runs of a raw file) are read with parallel preads into
// pinned host memory (the device's library-owned slot ring, or a caller's
// buffer), copied to the device in batches and decoded there.
//
// The reference reads the window with h5["data"][idxs...]
// (src/gbtworkerfunctions.jl:181-187): libhdf5 reads each chunk, H5Zbitshuffle
// (Project.toml:10) decompresses it on the host, libhdf5 assembles the
// hyperslab.  Here only compressed bytes cross PCIe and the decode runs on the
// GPU; the window is then a view of, or a gather from, the decoded chunk grid
// (fbh5.py).  Everything up to the GPU queue is native C++ threads, so the
// reads never wait on the Python interpreter lock:
//   * a persistent pool of reader threads pulls pread pieces in batch order
//     (adjacent chunks merged into runs, runs cut into pieces);
//   * the calling thread waits for each batch's pieces, queues its H2D copy on
//     `copy_stream`, makes `stream` wait for it and queues the batch's decode
//     (bldp_bslz4_decode_dev_async) or raw-chunk copies on `stream`.
// Batch b+1 is being read while batch b is copied and decoded.  The reader
// threads run on the CPUs of the GPU's NUMA node and the slots sit on that
// node (round 5: the page-cache copies stay on the GPU's socket and leave
// CPU quota to the caller; profiles/r05/reads/).
#include <errno.h>
#include <pthread.h>
#include <sched.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cctype>
#include <condition_variable>
#include <cstdio>
#include <cstring>
#include <cstdlib>
#include <map>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#include "bldp_impl.h"

namespace {

struct Piece {
  int64_t foff, hoff, len;
  int32_t batch;
  int32_t fd;  // -1 = the job's fd
};

// One call's reads.  `left[b]` counts the pieces of batch b still unread.
// Pieces land at host + hoff, or, with a slot ring, in slot (batch % nslot)
// at hoff - batch * slot_bytes; then only batches below `open` may be read
// (their slot's previous copy is done).
//
// Copy-out jobs (bldp_device_to_host) use the same pieces the other way
// round: `copy_src` is the slot ring, a piece of batch b is a memcpy from
// slot b % nslot to host + hoff, and `open` counts the batches whose DMA into
// their slot has landed.
struct Job {
  int fd = -1;
  uint8_t *host = nullptr;
  const std::vector<void *> *slot_base = nullptr;
  const std::vector<void *> *copy_src = nullptr;
  int64_t slot_bytes = 0;
  // slot ring with batches of any size (the chunk reader): batch b starts at
  // staged offset batch_lo[b], i.e. at the start of its slot; empty: batch b
  // starts at b * slot_bytes
  std::vector<int64_t> batch_lo;
  std::vector<Piece> pieces;
  std::unique_ptr<std::atomic<int64_t>[]> left;
  std::atomic<int64_t> next{0};
  std::atomic<int64_t> open{INT64_MAX};
  std::atomic<int> err{0};
  std::mutex mu;
  std::condition_variable cv, gate;
};

// The CPUs of device `dev`'s NUMA node that this process may run on (the
// node of the GPU's PCIe root, where the pinned slots the readers fill should
// be copied from and to); false when the node or its CPU list is unknown.
int device_numa_node(int dev) {
  char bus[64] = {0};
  if (hipDeviceGetPCIBusId(bus, (int)sizeof(bus), dev) != hipSuccess) {
    (void)hipGetLastError();
    return -1;
  }
  for (char *c = bus; *c; ++c) *c = (char)tolower((unsigned char)*c);
  char path[160];
  snprintf(path, sizeof(path), "/sys/bus/pci/devices/%s/numa_node", bus);
  FILE *f = fopen(path, "r");
  if (!f) return -1;
  int node = -1;
  if (fscanf(f, "%d", &node) != 1) node = -1;
  fclose(f);
  return node;
}

bool device_node_cpus(int dev, cpu_set_t *set) {
  const int node = device_numa_node(dev);
  if (node < 0) return false;
  char path[160];
  snprintf(path, sizeof(path), "/sys/devices/system/node/node%d/cpulist", node);
  FILE *f = fopen(path, "r");
  if (!f) return false;
  cpu_set_t want;
  CPU_ZERO(&want);
  int lo = 0, hi = 0;
  char sep = 0;
  while (fscanf(f, "%d", &lo) == 1) {  // "0-63,128-191"
    hi = lo;
    if (fscanf(f, "%c", &sep) == 1 && sep == '-') {
      if (fscanf(f, "%d", &hi) != 1) break;
      if (fscanf(f, "%c", &sep) != 1) sep = 0;
    }
    for (int c = lo; c <= hi && c < CPU_SETSIZE; ++c) CPU_SET(c, &want);
    if (sep != ',') break;
  }
  fclose(f);
  cpu_set_t allowed;
  if (sched_getaffinity(0, sizeof(allowed), &allowed) != 0) return false;
  CPU_AND(set, &want, &allowed);
  return CPU_COUNT(set) > 0;
}

// Reader threads: 16, or 4 fewer than the CPUs the process may use when that
// is less (the cgroup's CPU quota, else the affinity mask), so the readers do
// not starve the calling thread and the HIP runtime's threads of their quota:
// on a 16-CPU quota 12 readers read a band 10-25% faster than 16 (round 5,
// profiles/r05/reads/).
int default_reader_threads() {
  int cpus = (int)std::thread::hardware_concurrency();
  cpu_set_t allowed;
  if (sched_getaffinity(0, sizeof(allowed), &allowed) == 0) cpus = CPU_COUNT(&allowed);
  long long quota = 0, period = 0;
  if (FILE *f = fopen("/sys/fs/cgroup/cpu.max", "r")) {  // cgroup v2: "quota period" or "max ..."
    if (fscanf(f, "%lld %lld", &quota, &period) != 2) quota = 0;
    fclose(f);
  } else if (FILE *q = fopen("/sys/fs/cgroup/cpu/cpu.cfs_quota_us", "r")) {  // cgroup v1
    if (fscanf(q, "%lld", &quota) != 1) quota = 0;
    fclose(q);
    if (FILE *p = fopen("/sys/fs/cgroup/cpu/cpu.cfs_period_us", "r")) {
      if (fscanf(p, "%lld", &period) != 1) period = 0;
      fclose(p);
    }
  }
  if (quota > 0 && period > 0) cpus = std::min<long long>(cpus, std::max<long long>(1, quota / period));
  return std::min(16, std::max(2, cpus >= 16 + 4 ? 16 : cpus - 4));
}

class ReadPool {
 public:
  // n reader threads, each confined to `cpus` when given
  explicit ReadPool(int n, const cpu_set_t *cpus = nullptr) {
    for (int i = 0; i < n; ++i) {
      th_.emplace_back([this] { work(); });
      if (cpus) (void)pthread_setaffinity_np(th_.back().native_handle(), sizeof(*cpus), cpus);
    }
  }
  ~ReadPool() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto &t : th_) t.join();
  }
  int threads() const { return (int)th_.size(); }
  // Publish `j`; its pieces are read by the pool (and by the caller's waits).
  void post(Job *j) {
    {
      std::lock_guard<std::mutex> lk(mu_);
      job_ = j;
      ++gen_;
    }
    cv_.notify_all();
  }
  // Withdraw the job and wait until no reader thread still holds it.
  void retire() {
    std::unique_lock<std::mutex> lk(mu_);
    job_ = nullptr;
    idle_.wait(lk, [&] { return busy_ == 0; });
  }

 private:
  void work() {
    uint64_t seen = 0;
    for (;;) {
      Job *j;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return stop_ || (job_ && gen_ != seen); });
        if (stop_) return;
        seen = gen_;
        j = job_;
        ++busy_;
      }
      run(j);
      {
        std::lock_guard<std::mutex> lk(mu_);
        --busy_;
      }
      idle_.notify_all();
    }
  }

 public:
  static void run(Job *j) {
    const int64_t n = (int64_t)j->pieces.size();
    for (;;) {
      const int64_t i = j->next.fetch_add(1);
      if (i >= n) return;
      const Piece &p = j->pieces[i];
      if (j->copy_src) {  // copy-out: slot -> caller memory once the batch's DMA landed
        if (p.batch >= j->open.load()) {
          std::unique_lock<std::mutex> lk(j->mu);
          j->gate.wait(lk, [&] { return p.batch < j->open.load() || j->err.load(); });
        }
        if (!j->err.load(std::memory_order_relaxed)) {
          const std::vector<void *> &sl = *j->copy_src;
          std::memcpy(j->host + p.hoff,
                      (const uint8_t *)sl[p.batch % sl.size()] + (p.hoff - p.batch * j->slot_bytes),
                      (size_t)p.len);
        }
        if (j->left[p.batch].fetch_sub(1) == 1 || j->err.load()) {
          std::lock_guard<std::mutex> lk(j->mu);
          j->cv.notify_all();
        }
        continue;
      }
      uint8_t *dst = j->host + p.hoff;
      if (j->slot_base) {
        if (p.batch >= j->open.load()) {  // wait for the slot
          std::unique_lock<std::mutex> lk(j->mu);
          j->gate.wait(lk, [&] { return p.batch < j->open.load() || j->err.load(); });
        }
        const std::vector<void *> &sl = *j->slot_base;
        const int64_t lo = j->batch_lo.empty() ? p.batch * j->slot_bytes : j->batch_lo[p.batch];
        dst = (uint8_t *)sl[p.batch % sl.size()] + (p.hoff - lo);
      }
      int64_t got = 0;
      while (got < p.len && !j->err.load(std::memory_order_relaxed)) {
        const ssize_t r = pread(p.fd >= 0 ? p.fd : j->fd, dst + got, (size_t)(p.len - got),
                                p.foff + got);
        if (r < 0 && errno == EINTR) continue;
        if (r <= 0) {
          int expect = 0;
          j->err.compare_exchange_strong(expect, r < 0 ? errno : EIO);
          break;
        }
        got += r;
      }
      if (j->left[p.batch].fetch_sub(1) == 1 || j->err.load()) {
        std::lock_guard<std::mutex> lk(j->mu);
        j->cv.notify_all();
      }
    }
  }

 private:
  std::vector<std::thread> th_;
  std::mutex mu_;
  std::condition_variable cv_, idle_;
  Job *job_ = nullptr;
  uint64_t gen_ = 0;
  int busy_ = 0;
  bool stop_ = false;
};

// nslot pinned host slots of `bytes` each (bldp_runs_to_device's ring).
// The chunk reader's default ring: 8 x 32 MiB, the geometry filestream.py
// gives bldp_runs_to_device, so the two readers share one ring per device.
constexpr int64_t kRingSlotBytes = 32ll << 20;
constexpr int kRingSlots = 8;
struct Slots {
  int64_t bytes = 0;
  std::vector<void *> p;
};

// Per device (the caller's current device): a pool of reader threads
// (BLDP_READ_THREADS, default 16), the slot ring and the lock that lets one
// read call at a time use them.  Reads for different GPUs (the GBT fan-out
// over several GPUs of a node) run side by side.
struct DevIO {
  std::mutex call;
  std::unique_ptr<ReadPool> pool;
  Slots slots;
  bool node_pinned = false;  // readers confined to the GPU's NUMA node
  int node = -1;             // the GPU's NUMA node (-1: unknown)
  bool retired = false;  // released by bldp_finalize (under `call`)
};
std::mutex g_io_mu;
std::map<int, std::shared_ptr<DevIO>> g_io;

// The current device's DevIO, returned with its call lock held in `call`.
// The shared_ptr keeps it alive across a concurrent fileio_release; one
// released while this thread waited for its call lock is retired, and the
// loop takes the fresh one instead.
std::shared_ptr<DevIO> dev_io(std::unique_lock<std::mutex> &call) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) dev = 0;
  for (;;) {
    std::shared_ptr<DevIO> io;
    {
      std::lock_guard<std::mutex> lk(g_io_mu);
      std::shared_ptr<DevIO> &slot = g_io[dev];
      if (!slot) {
        int n = 0;
        if (const char *e = getenv("BLDP_READ_THREADS")) n = atoi(e);
        if (n <= 0) n = default_reader_threads();
        slot = std::make_shared<DevIO>();
        // the readers run on the CPUs of the GPU's NUMA node (BLDP_READ_AFFINITY=0:
        // anywhere), so the page-cache copies into the pinned slots, which sit
        // on that node too (ensure_slots), stay on the GPU's socket
        cpu_set_t cpus;
        const char *aff = getenv("BLDP_READ_AFFINITY");
        // (only where that node has at least half as many allowed CPUs as
        // there are readers: 16 readers on the 1-2 node CPUs of a cpuset that
        // spans sockets would crowd them)
        const bool pin = !(aff && atoi(aff) == 0) && device_node_cpus(dev, &cpus) &&
                         2 * CPU_COUNT(&cpus) >= n;
        slot->pool.reset(new ReadPool(n, pin ? &cpus : nullptr));
        slot->node_pinned = pin;
        slot->node = device_numa_node(dev);
      }
      io = slot;
    }
    std::unique_lock<std::mutex> lk(io->call);
    if (!io->retired) {
      call = std::move(lk);
      return io;
    }
  }
}

double ms_since(std::chrono::steady_clock::time_point t0) {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

// A job published to a pool; whatever way the call leaves (error return or
// C++ exception), the readers are cancelled and withdrawn before the job (a
// local of the call) goes away.
struct PostedJob {
  ReadPool *rp;
  Job *j;
  bool done = false;
  PostedJob(ReadPool *r, Job *jj) : rp(r), j(jj) { rp->post(j); }
  void finish(bool cancel) {
    if (done) return;
    done = true;
    if (cancel) {
      {
        std::lock_guard<std::mutex> lk(j->mu);
        int expect = 0;
        j->err.compare_exchange_strong(expect, ECANCELED);
        j->open.store(INT64_MAX);
      }
      j->gate.notify_all();
      ReadPool::run(j);  // the remaining pieces, skipped
    }
    rp->retire();
  }
  ~PostedJob() { finish(true); }
};

// The ring reused across calls of one device (under its call lock).
void free_slots(Slots &sl) {
  for (void *q : sl.p) (void)hipHostFree(q);
  sl.p.clear();
  sl.bytes = 0;
}
// node >= 0: the slots' pages are placed on that NUMA node, the GPU's (the
// calling thread's memory policy set to prefer it while the runtime pins
// them, hipHostMallocNumaUser); BLDP_SLOT_NUMA=0: wherever the runtime puts
// them.
int ensure_slots(Slots &sl, int64_t bytes, int nslot, int node = -1) {
  if (sl.bytes == bytes && (int)sl.p.size() == nslot) return BLDP_OK;
  free_slots(sl);
  const char *e = getenv("BLDP_SLOT_NUMA");
  bool numa = node >= 0 && node < 64 && !(e && atoi(e) == 0);
  constexpr int kMpolDefault = 0, kMpolPreferred = 1;  // <numaif.h>, no libnuma
  // only a thread on the default policy is switched (and switched back to
  // it): a caller's own policy (numactl --membind / --interleave, or one it
  // set) stays in force and places the slots itself
  int prev_mode = -1;
  unsigned long prev_mask[16] = {0};
  if (numa && (syscall(SYS_get_mempolicy, &prev_mode, prev_mask, 16 * 64, nullptr, 0) != 0 ||
               prev_mode != kMpolDefault))
    numa = false;
  unsigned long mask = 1ul << (node >= 0 && node < 64 ? node : 0);
  if (numa && syscall(SYS_set_mempolicy, kMpolPreferred, &mask, 64) != 0) mask = 0;
  struct Restore {
    bool on;
    ~Restore() {
      if (on) (void)syscall(SYS_set_mempolicy, kMpolDefault, nullptr, 0);  // (was default)
    }
  } restore{numa && mask};
  const unsigned flags = restore.on ? hipHostMallocNumaUser : hipHostMallocDefault;
  for (int i = 0; i < nslot; ++i) {
    void *q = nullptr;
    if (hipHostMalloc(&q, (size_t)bytes, flags) != hipSuccess) {
      free_slots(sl);
      return bldp::set_error(BLDP_ENOMEM, "%lld bytes of pinned slots",
                             (long long)bytes);
    }
    sl.p.push_back(q);
  }
  sl.bytes = bytes;
  return BLDP_OK;
}

}  // namespace

// fds: one descriptor per chunk (the chunks of several files -- a band's banks
// -- in one stream of batches), or NULL: every chunk is in `fd`.
static int chunks_to_device(
    int fd, const int *fds, int64_t nchunk, const int64_t *file_off, const int64_t *stored_len,
    const int64_t *stage_off, const uint32_t *filter_mask, int64_t nbatch, const int64_t *batch_end,
    void *host_pinned, void *dev_stage, int64_t stage_bytes, void *dev_out, int64_t out_chunk_bytes,
    int64_t out_bytes, int *err_dev, void *copy_stream, void *stream, double *stats) {
  const auto t0 = std::chrono::steady_clock::now();
  if (nchunk < 0 || nbatch < 0 || (nchunk && (!file_off || !stored_len || !stage_off ||
                                               !filter_mask || !batch_end || !dev_stage ||
                                               nbatch < 1)))
    return bldp::set_error(BLDP_EINVAL, "chunks_to_device: bad argument");
  if (nchunk == 0) return BLDP_OK;
  if (batch_end[nbatch - 1] != nchunk)
    return bldp::set_error(BLDP_EINVAL, "chunks_to_device: batches must end at chunk %lld",
                           (long long)nchunk);
  bool any_comp = false;
  if (dev_out && (out_chunk_bytes < 0 || nchunk > out_bytes / std::max<int64_t>(1, out_chunk_bytes)))
    return bldp::set_error(BLDP_EINVAL, "chunks_to_device: %lld chunks of %lld bytes exceed the "
                           "%lld-byte output", (long long)nchunk, (long long)out_chunk_bytes,
                           (long long)out_bytes);
  for (int64_t k = 0; k < nchunk; ++k) {
    if (stored_len[k] < 0 || stage_off[k] < 0 || file_off[k] < 0)
      return bldp::set_error(BLDP_EINVAL, "chunks_to_device: negative offset or size");
    if (fds && stored_len[k] && fds[k] < 0)
      return bldp::set_error(BLDP_EINVAL, "chunks_to_device: chunk %lld has no file", (long long)k);
    if (stored_len[k] > stage_bytes - stage_off[k])
      return bldp::set_error(BLDP_EINVAL, "chunks_to_device: chunk %lld overruns the %lld-byte "
                             "staging buffers", (long long)k, (long long)stage_bytes);
    if (stored_len[k] && (filter_mask[k] & 1) && dev_out && stored_len[k] != out_chunk_bytes)
      return bldp::set_error(BLDP_EINVAL,
                             "chunks_to_device: unfiltered chunk %lld holds %lld bytes, not %lld",
                             (long long)k, (long long)stored_len[k], (long long)out_chunk_bytes);
    any_comp = any_comp || (stored_len[k] && !(filter_mask[k] & 1));
  }
  if (any_comp && (!dev_out || !err_dev))
    return bldp::set_error(BLDP_EINVAL, "chunks_to_device: compressed chunks need an output");

  // pieces: per batch, chunks adjacent in the file and in the staging buffer
  // merge into runs; a batch of <= 32 MiB is cut into ~16 pieces (the whole
  // pool reads it), larger ones into ~8
  Job j;
  j.fd = fd;
  j.host = (uint8_t *)host_pinned;
  j.left.reset(new std::atomic<int64_t>[nbatch]);
  std::vector<std::pair<int64_t, int64_t>> brange(nbatch);  // staged byte range of a batch
  int64_t k0 = 0;
  for (int64_t b = 0; b < nbatch; ++b) {
    const int64_t k1 = batch_end[b];
    if (k1 < k0 || k1 > nchunk)
      return bldp::set_error(BLDP_EINVAL, "chunks_to_device: batch ends out of order");
    int64_t lo = INT64_MAX, hi = 0, bytes = 0;
    for (int64_t k = k0; k < k1; ++k)
      if (stored_len[k]) {
        lo = std::min(lo, stage_off[k]);
        hi = std::max(hi, stage_off[k] + stored_len[k]);
        bytes += stored_len[k];
      }
    brange[b] = {lo == INT64_MAX ? 0 : lo, hi};
    const int64_t piece =
        std::max<int64_t>(256 << 10, bytes <= (32ll << 20) ? bytes / 16 : bytes / 8);
    const size_t first = j.pieces.size();
    for (int64_t k = k0; k < k1;) {
      if (!stored_len[k]) {
        ++k;
        continue;
      }
      int64_t f = file_off[k], h = stage_off[k], n = stored_len[k];
      const int kfd = fds ? fds[k] : -1;
      int64_t q = k + 1;
      while (q < k1 && stored_len[q] && file_off[q] == f + n && stage_off[q] == h + n &&
             (!fds || fds[q] == kfd)) {
        n += stored_len[q];
        ++q;
      }
      for (int64_t x = 0; x < n; x += piece)
        j.pieces.push_back({f + x, h + x, std::min(piece, n - x), (int32_t)b, kfd});
      k = q;
    }
    j.left[b].store((int64_t)(j.pieces.size() - first));
    k0 = k1;
  }

  // every buffer of the queueing loop is allocated before the readers start
  int64_t maxb = 0;
  for (int64_t b = 0, q = 0; b < nbatch; q = batch_end[b], ++b)
    maxb = std::max(maxb, batch_end[b] - q);
  std::vector<hipEvent_t> evs(nbatch, nullptr);  // batch b's H2D copy done
  std::vector<uint64_t> offs, lens, ooff, olen;
  for (auto *v : {&offs, &lens, &ooff, &olen}) v->reserve(maxb);
  std::unique_lock<std::mutex> call;
  const std::shared_ptr<DevIO> io = dev_io(call);
  ReadPool *rp = io->pool.get();
  // host_pinned NULL: batch b is read into slot b % nslot of the device's
  // pinned ring (the one bldp_runs_to_device uses, kept when its slots hold
  // the largest batch), reopened once the slot's previous H2D copy is done
  const bool ring = host_pinned == nullptr;
  int64_t nslot = 0;
  if (ring) {
    int64_t span = 0;
    for (const auto &r : brange) span = std::max(span, r.second - r.first);
    if (io->slots.p.size() < 2 || io->slots.bytes < span) {
      int nring = kRingSlots;  // (BLDP_RING_SLOTS: a probe knob, 2..16)
      if (const char *e = getenv("BLDP_RING_SLOTS")) nring = std::min(16, std::max(2, atoi(e)));
      // a batch larger than a ring slot (one big unfiltered chunk): two slots
      // of its size, released when the call returns (the ring
      // stays bounded between calls whatever the chunk size)
      if (span > kRingSlotBytes) nring = 2;
      const int rc = ensure_slots(io->slots, std::max(kRingSlotBytes, (span + (1 << 20) - 1) &
                                                                          ~(int64_t)((1 << 20) - 1)),
                                  nring, io->node);
      if (rc) return rc;
    }
    nslot = (int64_t)io->slots.p.size();
    j.slot_base = &io->slots.p;
    j.slot_bytes = io->slots.bytes;
    j.batch_lo.resize(nbatch);
    for (int64_t b = 0; b < nbatch; ++b) j.batch_lo[b] = brange[b].first;
    j.open.store(std::min<int64_t>(nbatch, nslot));
  }
  PostedJob posted(rp, &j);
  hipStream_t cs = (hipStream_t)copy_stream, s = (hipStream_t)stream;
  int rc = BLDP_OK;
  double t_first = -1.0;
  k0 = 0;
  for (int64_t b = 0; b < nbatch && rc == BLDP_OK; ++b) {
    const int64_t k1 = batch_end[b];
    {  // this batch's reads
      std::unique_lock<std::mutex> lk(j.mu);
      j.cv.wait(lk, [&] { return j.left[b].load() == 0 || j.err.load(); });
    }
    if (int e = j.err.load()) {
      rc = bldp::set_error(BLDP_EIO, "chunks_to_device: read failed (%s): truncated file or "
                           "stale chunk index?", strerror(e));
      break;
    }
    const int64_t lo = brange[b].first, hi = brange[b].second;
    // the batch's staged bytes on the host, and the offset they start at
    const uint8_t *hsrc = ring ? (const uint8_t *)io->slots.p[b % nslot] : (const uint8_t *)host_pinned + lo;
    if (hi > lo) {
      if (hipEventCreateWithFlags(&evs[b], hipEventDisableTiming) != hipSuccess) {
        rc = bldp::set_error(BLDP_EHIP, "chunks_to_device: event create failed");
        break;
      }
      hipEvent_t ev = evs[b];
      if (hipMemcpyAsync((uint8_t *)dev_stage + lo, hsrc, (size_t)(hi - lo),
                         hipMemcpyHostToDevice, cs) != hipSuccess ||
          hipEventRecord(ev, cs) != hipSuccess || hipStreamWaitEvent(s, ev, 0) != hipSuccess) {
        rc = bldp::set_error(BLDP_EHIP, "chunks_to_device: H2D copy of batch %lld failed",
                             (long long)b);
        break;
      }
      if (t_first < 0) t_first = ms_since(t0);
    }
    offs.clear();
    lens.clear();
    ooff.clear();
    olen.clear();
    for (int64_t k = k0; k < k1 && rc == BLDP_OK; ++k) {
      if (!stored_len[k]) continue;
      if (filter_mask[k] & 1) {  // stored without the filter: raw elements
        if (dev_out && hipMemcpyAsync((uint8_t *)dev_out + k * out_chunk_bytes,
                                      (uint8_t *)dev_stage + stage_off[k],
                                      (size_t)out_chunk_bytes, hipMemcpyDeviceToDevice,
                                      s) != hipSuccess)
          rc = bldp::set_error(BLDP_EHIP, "chunks_to_device: raw chunk copy failed");
        continue;
      }
      offs.push_back((uint64_t)stage_off[k]);
      lens.push_back((uint64_t)stored_len[k]);
      ooff.push_back((uint64_t)(k * out_chunk_bytes));
      olen.push_back((uint64_t)out_chunk_bytes);
    }
    // (the decoder reads each chunk's 12-byte header on the host, here: before
    // the batch's slot can be reopened below)
    if (rc == BLDP_OK && !offs.empty())
      rc = bldp::bslz4_decode_async_at((int)offs.size(), hsrc, (uint64_t)lo,
                                       (const uint8_t *)dev_stage, offs.data(), lens.data(), 4,
                                       (uint8_t *)dev_out, ooff.data(), olen.data(), err_dev, s);
    if (rc == BLDP_OK && ring && b >= 1) {  // slot of batch b - 1: free once its copy is done
      if (evs[b - 1] && hipEventSynchronize(evs[b - 1]) != hipSuccess) {
        rc = bldp::set_error(BLDP_EHIP, "chunks_to_device: copy of batch %lld failed",
                             (long long)(b - 1));
        break;
      }
      {
        std::lock_guard<std::mutex> lk(j.mu);
        j.open.store(std::min<int64_t>(nbatch, b - 1 + nslot + 1));
      }
      j.gate.notify_all();
    }
    k0 = k1;
  }
  const double t_reads = ms_since(t0);
  posted.finish(rc != BLDP_OK);  // (an error: cancel the readers first)
  // the ring's slots are reused by the next call: no copy out of them may
  // outlive this one (the caller's buffer: bldp_bslz4_error waits instead)
  for (hipEvent_t ev : evs)
    if (ev) {
      if (ring && hipEventSynchronize(ev) != hipSuccess && rc == BLDP_OK)
        rc = bldp::set_error(BLDP_EHIP, "chunks_to_device: copy failed");
      (void)hipEventDestroy(ev);
    }
  if (ring && io->slots.bytes > kRingSlotBytes) free_slots(io->slots);  // (oversized batches)
  if (stats) {
    stats[0] = t_first;
    stats[1] = t_reads;
    stats[2] = (double)j.pieces.size();
    stats[3] = (double)rp->threads();
  }
  return rc;
}

// ---------------------------------------------------------------------------
// Raw runs (uncompressed contiguous FBH5 `data`, SIGPROC data blocks) into a
// dense device block through a ring of library-owned pinned slots.
// fds: one descriptor per run (runs of several files in one stream of
// batches), or NULL: every run is in `fd`.
static int runs_to_device(int fd, const int *fds, int64_t nrun, const int64_t *file_off,
                          const int64_t *len, void *dev_dst, int64_t dst_bytes,
                          int64_t slot_bytes, int nslot, void *copy_stream, void *stream,
                          double *stats) {
  const auto t0 = std::chrono::steady_clock::now();
  if (nrun < 0 || (nrun && (!file_off || !len || !dev_dst)) || slot_bytes < (1 << 20) ||
      nslot < 2 || nslot > 16)
    return bldp::set_error(BLDP_EINVAL, "runs_to_device: bad argument");
  int64_t total = 0;
  for (int64_t r = 0; r < nrun; ++r) {
    if (len[r] < 0 || file_off[r] < 0)
      return bldp::set_error(BLDP_EINVAL, "runs_to_device: negative offset or size");
    if (fds && fds[r] < 0 && len[r] > 0)
      return bldp::set_error(BLDP_EINVAL, "runs_to_device: run %lld has no file", (long long)r);
    total += len[r];
  }
  if (total > dst_bytes)
    return bldp::set_error(BLDP_EINVAL, "runs_to_device: %lld bytes exceed the %lld-byte "
                           "destination", (long long)total, (long long)dst_bytes);
  if (total == 0) return BLDP_OK;
  // batches: slot-sized, but (blocks of more than 4 slots) the first two and
  // the last two ramp (slot/4, slot/2 ... slot/2, slot/4), so the first copy
  // starts after a quarter slot of reads and the copy left after the last
  // read is a quarter slot (BLDP_RUNS_RAMP=0: uniform, a probe knob)
  std::vector<int64_t> blo;  // batch b = [blo[b], blo[b + 1])
  {
    const char *e = getenv("BLDP_RUNS_RAMP");
    const bool ramp = !(e && atoi(e) == 0) && total > 4 * slot_bytes;
    const int64_t q = std::max<int64_t>(1 << 20, slot_bytes / 4);
    const int64_t h = std::max<int64_t>(1 << 20, slot_bytes / 2);
    int64_t at = 0, mid_end = total;
    blo.push_back(0);
    if (ramp) {
      blo.push_back(at += q);
      blo.push_back(at += h);
      mid_end = total - h - q;
    }
    while (at < mid_end) blo.push_back(at = std::min(at + slot_bytes, mid_end));
    if (ramp) {
      blo.push_back(at += h);
      blo.push_back(at += q);
    }
  }
  const int64_t nbatch = (int64_t)blo.size() - 1;
  // pieces: runs cut at batch boundaries and into ~8 pieces per batch;
  // piece.hoff is the offset in the whole block (the slot is batch % nslot)
  Job j;
  j.fd = fd;
  j.left.reset(new std::atomic<int64_t>[nbatch]);
  for (int64_t b = 0; b < nbatch; ++b) j.left[b].store(0);
  int64_t pos = 0, b = 0;
  for (int64_t r = 0; r < nrun; ++r) {
    int64_t x = 0;
    while (x < len[r]) {
      while (pos + x >= blo[b + 1]) ++b;
      const int64_t piece = std::max<int64_t>(256 << 10, (blo[b + 1] - blo[b]) / 8);
      const int64_t n = std::min({piece, len[r] - x, blo[b + 1] - (pos + x)});
      j.pieces.push_back({file_off[r] + x, pos + x, n, (int32_t)b, fds ? fds[r] : -1});
      j.left[b].fetch_add(1);
      x += n;
    }
    pos += len[r];
  }
  std::unique_lock<std::mutex> call;
  const std::shared_ptr<DevIO> io = dev_io(call);
  int rc = ensure_slots(io->slots, slot_bytes, nslot, io->node);
  if (rc) return rc;
  // reads of batch b go to slot b % nslot at (hoff - blo[b]); a batch may be
  // read once the copy out of its slot one round back is done
  j.slot_base = &io->slots.p;
  j.slot_bytes = slot_bytes;
  j.batch_lo.assign(blo.begin(), blo.end() - 1);
  j.open.store(std::min<int64_t>(nbatch, nslot));
  std::vector<hipEvent_t> evs(nbatch, nullptr);
  ReadPool *rp = io->pool.get();
  PostedJob posted(rp, &j);
  hipStream_t cs = (hipStream_t)copy_stream, s = (hipStream_t)stream;
  double t_first = -1.0;
  for (int64_t b = 0; b < nbatch && rc == BLDP_OK; ++b) {
    {
      std::unique_lock<std::mutex> lk(j.mu);
      j.cv.wait(lk, [&] { return j.left[b].load() == 0 || j.err.load(); });
    }
    if (int e = j.err.load()) {
      rc = bldp::set_error(BLDP_EIO, "runs_to_device: read failed (%s): truncated file?",
                           strerror(e));
      break;
    }
    const int64_t lo = blo[b], n = blo[b + 1] - lo;
    if (hipEventCreateWithFlags(&evs[b], hipEventDisableTiming) != hipSuccess ||
        hipMemcpyAsync((uint8_t *)dev_dst + lo, io->slots.p[b % nslot], (size_t)n,
                       hipMemcpyHostToDevice, cs) != hipSuccess ||
        hipEventRecord(evs[b], cs) != hipSuccess) {
      rc = bldp::set_error(BLDP_EHIP, "runs_to_device: H2D copy of batch %lld failed",
                           (long long)b);
      break;
    }
    if (t_first < 0) t_first = ms_since(t0);
    if (b >= 1) {  // the slot of batch b - 1 is free once its copy is done
      if (hipEventSynchronize(evs[b - 1]) != hipSuccess) {
        rc = bldp::set_error(BLDP_EHIP, "runs_to_device: copy of batch %lld failed",
                             (long long)(b - 1));
        break;
      }
      {
        std::lock_guard<std::mutex> lk(j.mu);
        j.open.store(std::min<int64_t>(nbatch, b - 1 + nslot + 1));
      }
      j.gate.notify_all();
    }
  }
  const double t_reads = ms_since(t0);
  posted.finish(rc != BLDP_OK);  // (an error: cancel the readers first)
  // the slots are reused by the next call: every copy out of them is done
  // before returning; the caller's stream waits for the last one
  for (int64_t b = 0; b < nbatch; ++b)
    if (evs[b]) {
      if (hipEventSynchronize(evs[b]) != hipSuccess && rc == BLDP_OK)
        rc = bldp::set_error(BLDP_EHIP, "runs_to_device: copy failed");
    }
  if (rc == BLDP_OK && evs[nbatch - 1] && hipStreamWaitEvent(s, evs[nbatch - 1], 0) != hipSuccess)
    rc = bldp::set_error(BLDP_EHIP, "runs_to_device: stream wait failed");
  for (hipEvent_t ev : evs)
    if (ev) (void)hipEventDestroy(ev);
  if (stats) {
    stats[0] = t_first;
    stats[1] = t_reads;
    stats[2] = (double)j.pieces.size();
    stats[3] = (double)rp->threads();
  }
  return rc;
}

extern "C" BLDP_API int bldp_chunks_to_device(
    int fd, int64_t nchunk, const int64_t *file_off, const int64_t *stored_len,
    const int64_t *stage_off, const uint32_t *filter_mask, int64_t nbatch, const int64_t *batch_end,
    void *host_pinned, void *dev_stage, int64_t stage_bytes, void *dev_out, int64_t out_chunk_bytes,
    int64_t out_bytes, int *err_dev, void *copy_stream, void *stream, double *stats) {
  try {
    return chunks_to_device(fd, nullptr, nchunk, file_off, stored_len, stage_off, filter_mask,
                            nbatch, batch_end, host_pinned, dev_stage, stage_bytes, dev_out,
                            out_chunk_bytes, out_bytes, err_dev, copy_stream, stream, stats);
  } catch (const std::bad_alloc &) {
    return bldp::set_error(BLDP_ENOMEM, "chunks_to_device: out of host memory");
  } catch (...) {
    return bldp::set_error(BLDP_EINVAL, "chunks_to_device: unexpected C++ exception");
  }
}

extern "C" BLDP_API int bldp_file_chunks_to_device(
    int64_t nchunk, const int *fd, const int64_t *file_off, const int64_t *stored_len,
    const int64_t *stage_off, const uint32_t *filter_mask, int64_t nbatch, const int64_t *batch_end,
    void *host_pinned, void *dev_stage, int64_t stage_bytes, void *dev_out, int64_t out_chunk_bytes,
    int64_t out_bytes, int *err_dev, void *copy_stream, void *stream, double *stats) {
  if (nchunk > 0 && !fd) return bldp::set_error(BLDP_EINVAL, "chunks_to_device: null fd array");
  try {
    return chunks_to_device(-1, fd, nchunk, file_off, stored_len, stage_off, filter_mask, nbatch,
                            batch_end, host_pinned, dev_stage, stage_bytes, dev_out,
                            out_chunk_bytes, out_bytes, err_dev, copy_stream, stream, stats);
  } catch (const std::bad_alloc &) {
    return bldp::set_error(BLDP_ENOMEM, "chunks_to_device: out of host memory");
  } catch (...) {
    return bldp::set_error(BLDP_EINVAL, "chunks_to_device: unexpected C++ exception");
  }
}

extern "C" BLDP_API int bldp_runs_to_device(int fd, int64_t nrun, const int64_t *file_off,
                                            const int64_t *len, void *dev_dst, int64_t dst_bytes,
                                            int64_t slot_bytes, int nslot, void *copy_stream,
                                            void *stream, double *stats) {
  try {
    return runs_to_device(fd, nullptr, nrun, file_off, len, dev_dst, dst_bytes, slot_bytes,
                          nslot, copy_stream, stream, stats);
  } catch (const std::bad_alloc &) {
    return bldp::set_error(BLDP_ENOMEM, "runs_to_device: out of host memory");
  } catch (...) {
    return bldp::set_error(BLDP_EINVAL, "runs_to_device: unexpected C++ exception");
  }
}

extern "C" BLDP_API int bldp_file_runs_to_device(int64_t nrun, const int *fd,
                                                 const int64_t *file_off, const int64_t *len,
                                                 void *dev_dst, int64_t dst_bytes,
                                                 int64_t slot_bytes, int nslot, void *copy_stream,
                                                 void *stream, double *stats) {
  if (nrun > 0 && !fd) return bldp::set_error(BLDP_EINVAL, "runs_to_device: null fd array");
  try {
    return runs_to_device(-1, fd, nrun, file_off, len, dev_dst, dst_bytes, slot_bytes, nslot,
                          copy_stream, stream, stats);
  } catch (const std::bad_alloc &) {
    return bldp::set_error(BLDP_ENOMEM, "runs_to_device: out of host memory");
  } catch (...) {
    return bldp::set_error(BLDP_EINVAL, "runs_to_device: unexpected C++ exception");
  }
}

// ---------------------------------------------------------------------------
// Device -> pageable host memory through the same pinned slot ring: the DMA
// of batch b + 1 runs while the reader threads copy batch b out of its slot.
// (GBT.getband's one device -> host copy of the stitched band, src/gbt.jl:103:
// the product lands in ordinary memory the caller owns, and no pinned memory
// is allocated or held per call.)
namespace {
constexpr int64_t kD2hSlotBytes = 32ll << 20;
constexpr int kD2hSlots = 8;
}  // namespace

static int device_to_host(const void *src, void *dst, int64_t bytes, void *copy_stream,
                          void *stream, double *stats) {
  const auto t0 = std::chrono::steady_clock::now();
  if (bytes < 0 || (bytes > 0 && (!src || !dst)))
    return bldp::set_error(BLDP_EINVAL, "device_to_host: bad argument");
  if (bytes == 0) return BLDP_OK;
  std::unique_lock<std::mutex> call;
  const std::shared_ptr<DevIO> io = dev_io(call);
  // the ring the file readers left (any slot size), else the default one
  int rc = io->slots.p.size() >= 2 ? BLDP_OK : ensure_slots(io->slots, kD2hSlotBytes, kD2hSlots, io->node);
  if (rc) return rc;
  // batches of up to a slot; a transfer of less than 4 slots is cut into 4
  // (>= 1 MiB each) so the DMA of one batch overlaps the copy-out of the
  // previous, and each batch into about two pieces per reader thread so the
  // whole pool copies it out (a 9 MB band product: 0.5 ms as 3 pieces of one
  // 9 MB batch)
  const int64_t nslot = (int64_t)io->slots.p.size();
  const int64_t sb = std::min<int64_t>(io->slots.bytes,
                                       std::max<int64_t>(1 << 20, ((bytes + 3) / 4 + 65535) & ~65535ll));
  const int64_t nbatch = (bytes + sb - 1) / sb;
  const int64_t piece =
      std::max<int64_t>(128 << 10, ((sb / (2 * io->pool->threads()) + 4095) & ~4095ll));
  Job j;
  j.host = (uint8_t *)dst;
  j.copy_src = &io->slots.p;
  j.slot_bytes = sb;  // (batch b: slot b % nslot from its start, sb <= the slot size)
  j.open.store(0);
  j.left.reset(new std::atomic<int64_t>[nbatch]);
  for (int64_t b = 0; b < nbatch; ++b) {
    const int64_t lo = b * sb, n = std::min(sb, bytes - lo);
    int64_t cnt = 0;
    for (int64_t x = 0; x < n; x += piece, ++cnt)
      j.pieces.push_back({0, lo + x, std::min(piece, n - x), (int32_t)b, -1});
    j.left[b].store(cnt);
  }
  hipStream_t cs = (hipStream_t)copy_stream, s = (hipStream_t)stream;
  hipEvent_t after = nullptr;  // the producer's work queued so far on `stream`
  std::vector<hipEvent_t> evs(nbatch, nullptr);
  if (hipEventCreateWithFlags(&after, hipEventDisableTiming) != hipSuccess ||
      hipEventRecord(after, s) != hipSuccess || hipStreamWaitEvent(cs, after, 0) != hipSuccess) {
    if (after) (void)hipEventDestroy(after);
    return bldp::set_error(BLDP_EHIP, "device_to_host: stream ordering failed");
  }
  ReadPool *rp = io->pool.get();
  double t_first = -1.0;
  {
    PostedJob posted(rp, &j);
    auto land = [&](int64_t b) -> bool {  // batch b's DMA done: open it for copy-out
      if (hipEventSynchronize(evs[b]) != hipSuccess) return false;
      {
        std::lock_guard<std::mutex> lk(j.mu);
        j.open.store(b + 1);
      }
      j.gate.notify_all();
      return true;
    };
    for (int64_t b = 0; b < nbatch && rc == BLDP_OK; ++b) {
      if (b >= nslot) {  // slot b % nslot: batch b - nslot copied out of it
        std::unique_lock<std::mutex> lk(j.mu);
        j.cv.wait(lk, [&] { return j.left[b - nslot].load() == 0 || j.err.load(); });
      }
      const int64_t lo = b * sb, n = std::min(sb, bytes - lo);
      if (hipEventCreateWithFlags(&evs[b], hipEventDisableTiming) != hipSuccess ||
          hipMemcpyAsync(io->slots.p[b % nslot], (const uint8_t *)src + lo, (size_t)n,
                         hipMemcpyDeviceToHost, cs) != hipSuccess ||
          hipEventRecord(evs[b], cs) != hipSuccess) {
        rc = bldp::set_error(BLDP_EHIP, "device_to_host: copy of batch %lld failed", (long long)b);
        break;
      }
      if (t_first < 0) t_first = ms_since(t0);
      if (b >= 1 && !land(b - 1))
        rc = bldp::set_error(BLDP_EHIP, "device_to_host: copy of batch %lld failed",
                             (long long)(b - 1));
    }
    if (rc == BLDP_OK && !land(nbatch - 1))
      rc = bldp::set_error(BLDP_EHIP, "device_to_host: copy of the last batch failed");
    if (rc == BLDP_OK) {
      ReadPool::run(&j);  // help with the last pieces, then wait for every one
      std::unique_lock<std::mutex> lk(j.mu);
      j.cv.wait(lk, [&] {
        for (int64_t b = 0; b < nbatch; ++b)
          if (j.left[b].load()) return false;
        return true;
      });
    }
    posted.finish(rc != BLDP_OK);
  }
  // no DMA into the slots may outlive the call (the next call reuses them)
  for (hipEvent_t ev : evs)
    if (ev) {
      (void)hipEventSynchronize(ev);
      (void)hipEventDestroy(ev);
    }
  (void)hipEventDestroy(after);
  if (stats) {
    stats[0] = t_first;
    stats[1] = ms_since(t0);
    stats[2] = (double)nbatch;
    stats[3] = (double)rp->threads();
  }
  return rc;
}

extern "C" BLDP_API int bldp_device_to_host(const void *src, void *dst, int64_t bytes,
                                            void *copy_stream, void *stream, double *stats) {
  try {
    return device_to_host(src, dst, bytes, copy_stream, stream, stats);
  } catch (const std::bad_alloc &) {
    return bldp::set_error(BLDP_ENOMEM, "device_to_host: out of host memory");
  } catch (...) {
    return bldp::set_error(BLDP_EINVAL, "device_to_host: unexpected C++ exception");
  }
}

void bldp::fileio_release() {
  std::lock_guard<std::mutex> lk(g_io_mu);
  for (auto &kv : g_io) {
    std::lock_guard<std::mutex> call(kv.second->call);  // no read call in progress
    kv.second->pool.reset();                            // joins the reader threads
    free_slots(kv.second->slots);
    kv.second->retired = true;  // a caller already holding it takes a fresh one
  }
  g_io.clear();
}
