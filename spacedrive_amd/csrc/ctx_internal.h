// ctx_internal.h — the sd_cas_ctx object and the host helpers shared by the C-ABI
// translation units (sd_hip_cas.cpp, host_paths.cpp, validator_host.cpp, sd_multi.cpp).  Not
// part of the public ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <dirent.h>
#include <pthread.h>
#include <sched.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/sd_hip_cas.h"

struct DevBuf {
  void* p = nullptr;
  size_t bytes = 0;
};

// Persistent host workers for the I/O gather (a 100-file job step cannot afford to spawn
// threads per call).  run(k, fn) executes fn on the caller plus k-1 pool threads and
// returns when all are done; fn pulls work items itself (atomic cursor).
class HostPool {
 public:
  // Round 6: the pool's threads may be confined to a CPU set — the CPUs of the GPU's NUMA
  // node (sd_cas_ctx_create), so the gather's page-cache copies and the pinned staging stay
  // on the socket whose PCIe root the DMA reads from.  Empty = the process's own mask.
  void set_cpus(const cpu_set_t& cpus, int ncpus) {
    std::lock_guard<std::mutex> g(mu_);
    cpus_ = cpus;
    ncpus_ = ncpus;
    for (auto& t : th_) (void)pthread_setaffinity_np(t.native_handle(), sizeof cpus_, &cpus_);
  }
  int bound_cpus() const { return ncpus_; }
  // Round 6: each pool thread may start by unsharing the process's descriptor table
  // (unshare(CLONE_FILES): a private copy of the table as it is then).  The readers open and
  // close a file per item, and with one shared table every open / close takes the same
  // table lock: 16 readers of config 1's mix gathered 575 k files/s shared and 745-775 k
  // private (tools/probe_gather.cpp, profiles/r06/gather/).  The rule this imposes: a pool
  // thread only uses descriptors it opened itself (or that existed when it started: the HIP
  // runtime's) — no task may hand a pool thread a descriptor opened elsewhere.  Set before
  // the first run (threads start lazily); SD_CAS_POOL_PRIVATE_FDS=0 keeps the shared table.
  // The copy would also keep every other descriptor of the process alive in this thread (a
  // pipe's write end: its reader never sees EOF; a socket the application closed: its peer
  // never sees the close; a dmabuf: its memory), so the thread then closes all of its copies
  // except 0-2 and what the HIP runtime holds — /dev/kfd, /dev/dri/renderD*, one eventfd
  // (tools/fd_list.py on the box: nothing else after HIP init, a context and a gather).
  void set_private_fds(bool on) { private_fds_ = on; }
  int private_threads() const { return nprivate_.load(); }
  ~HostPool() {
    {
      std::lock_guard<std::mutex> g(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : th_) t.join();
  }
  void run(unsigned k, const std::function<void()>& fn) {
    if (k <= 1) { fn(); return; }
    run2(k - 1, fn, fn);
  }
  // `workers` pool threads run fn while the caller runs caller_fn; returns when all are done
  void run2(unsigned workers, const std::function<void()>& fn, const std::function<void()>& caller_fn) {
    std::unique_lock<std::mutex> lk(mu_);
    while (th_.size() < workers) {
      th_.emplace_back([this] { loop(); });
      if (ncpus_) (void)pthread_setaffinity_np(th_.back().native_handle(), sizeof cpus_, &cpus_);
    }
    fn_ = &fn;
    want_ = workers;
    pending_ = workers;
    ++gen_;
    lk.unlock();
    cv_.notify_all();
    caller_fn();
    lk.lock();
    done_.wait(lk, [this] { return pending_ == 0; });
    fn_ = nullptr;
  }

 private:
  static void keep_only_device_fds() {
    DIR* d = opendir("/proc/thread-self/fd");
    if (!d) return;
    const int self = dirfd(d);
    std::vector<int> drop;
    char path[64], link[256];
    while (dirent* e = readdir(d)) {
      if (e->d_name[0] < '0' || e->d_name[0] > '9') continue;
      const int fd = atoi(e->d_name);
      if (fd == self || fd <= 2) continue;  // stdin/out/err stay (logging from a pool thread)
      snprintf(path, sizeof path, "/proc/thread-self/fd/%d", fd);
      const ssize_t n = readlink(path, link, sizeof link - 1);
      if (n < 0) continue;
      link[n] = 0;
      if (!strcmp(link, "/dev/kfd") || !strncmp(link, "/dev/dri/", 9) || !strcmp(link, "anon_inode:[eventfd]"))
        continue;
      drop.push_back(fd);
    }
    closedir(d);
    for (int fd : drop) close(fd);
  }
  void loop() {
    // private only where the copy can be swept (/proc mounted); closing a copy never releases
    // the application's POSIX locks (their owner is the table they were taken through)
    if (private_fds_ && access("/proc/thread-self/fd", R_OK) == 0 && unshare(CLONE_FILES) == 0) {
      keep_only_device_fds();
      nprivate_.fetch_add(1);
    }
    uint64_t seen = 0;
    std::unique_lock<std::mutex> lk(mu_);
    for (;;) {
      cv_.wait(lk, [&] { return stop_ || (gen_ != seen && want_ > 0); });
      if (stop_) return;
      seen = gen_;
      --want_;
      const std::function<void()>* f = fn_;
      lk.unlock();
      (*f)();
      lk.lock();
      if (--pending_ == 0) done_.notify_one();
    }
  }
  std::mutex mu_;
  std::condition_variable cv_, done_;
  std::vector<std::thread> th_;
  const std::function<void()>* fn_ = nullptr;
  unsigned want_ = 0, pending_ = 0;
  uint64_t gen_ = 0;
  bool stop_ = false;
  cpu_set_t cpus_{};
  int ncpus_ = 0;
  bool private_fds_ = false;
  std::atomic<int> nprivate_{0};
};

struct sd_cas_ctx {
  int device = 0;
  hipStream_t stream = nullptr;  // compute
  hipStream_t copy = nullptr;    // H2D side stream
  hipStream_t copy2 = nullptr;   // the streamed gather's early whole-file hash (A/B: pieces alternate)
  hipEvent_t copy2_done = nullptr;
  hipEvent_t h2d_done = nullptr;
  hipEvent_t packed_h2d = nullptr;   // the job step's whole-file pieces have landed (early hash)
  hipEvent_t packed_done = nullptr;  // ... and their hash (on copy2) has run
  DevBuf ws;       // kernel workspace
  DevBuf staging;  // device copy of a host batch
  DevBuf small;    // multi-device exchange buffers (sd_cas_multi_*)
  DevBuf cvbuf;    // file_checksum: one 32-B CV per 64 MiB segment
  DevBuf io;       // device copies of host arrays (sd_cas_identifier_links)
  void* pinned = nullptr;
  size_t pinned_bytes = 0;
  uint64_t* d_scalar = nullptr;  // 8 x u64 scratch for counters
  // the hash grouping's bucket totals: zero between calls (each call's last kernel re-zeroes
  // them), so the chain has no zeroing launch; ordered across streams like ws
  uint32_t* gtotals = nullptr;
  // The fused hash + group chain (sd_cas_hash_regions_sampled_dev / sd_cas_group_regions_dev):
  // two region sets used alternately, so set k's bucket tables can run on a side stream while
  // the next batch's K1G fills set k^1; region_done[k] orders set k's reuse after its tables.
  // gcursor holds both sets' cursors (2 x REGIONS u32, <= 1,024), zero between calls (the tables re-zero).
  uint32_t* gcursor = nullptr;
  DevBuf regions[2];
  uint64_t region_n[2] = {0, 0};
  const uint64_t* region_keys[2] = {nullptr, nullptr};  // the batch's keys (an overflowed region's regroup)
  hipEvent_t region_done[2] = {nullptr, nullptr};
  // recorded after set k's K1G: its tables (any stream) and its refill wait for it
  hipEvent_t region_hashed[2] = {nullptr, nullptr};
  bool region_pending[2] = {false, false};
  bool region_grouped[2] = {true, true};  // set k's tables have been enqueued since its K1G
  int region_cur = -1;
  // the Object counter of the last grouping call (d_scalar, or a region set's): what
  // sd_cas_copy_objects_dev copies; region_obj_set = that set (-1: d_scalar)
  int region_obj_set = -1;
  // ws and d_scalar are shared by every device call of the context, whatever stream the
  // caller passes: the last enqueued use is recorded here and a use on another stream
  // waits for it first (sd_ws_acquire / sd_ws_release)
  hipEvent_t ws_ev = nullptr;
  hipStream_t ws_stream = nullptr;
  bool ws_pending = false;
  size_t quantum = 65536;  // files per full wave of the device (CUs x 4 SIMDs x 64 lanes)
  int group_method = 0;       // SD_CAS_GROUP_* (sd_cas_set_group_method)
  uint64_t group_target = 0;  // mean keys per hash-grouping bucket (0 = tuned default)
  bool use_hash_group(uint64_t n) const {
    return group_method == SD_CAS_GROUP_HASH ||
           (group_method == SD_CAS_GROUP_AUTO && n <= SD_CAS_HASH_GROUP_MAX_KEYS);
  }
  // batches below these sizes use the chunk-parallel K1L kernel (sd_cas_set_latency_threshold)
  size_t latency_sampled = 0, latency_packed = 0;
  // K1L batches of at least this many files pack 4 files per wave (16-lane segments),
  // smaller ones take a wave per file (sd_cas_set_chunkpar_split)
  size_t seg16_sampled = 0, seg16_packed = 0;
  int chunkpar_seg(size_t n, bool sampled) const {
    return n >= (sampled ? seg16_sampled : seg16_packed) ? 16 : 64;
  }
  HostPool pool;  // I/O gather workers
  // the path gather's two window-slot events (persistent: creating them per call cost a
  // 100-file job step ~10 us)
  hipEvent_t gather_done[2] = {nullptr, nullptr};
  bool trace = false;  // SD_CAS_TRACE=1: per-phase host timestamps of host-buffer calls on stderr
  int numa_node = -1;  // the GPU's NUMA node (sysfs), -1 unknown; pool bound to it unless SD_CAS_POOL_NUMA=0
  uint32_t test_table_fill = 0;  // SD_CAS_TEST_TABLE_FILL (tests): region tables' overflow bound
  std::string err;
};

// Host phase timestamps of one blocking call (SD_CAS_TRACE=1): mark(name) after each phase,
// one stderr line at the end — "sd_cas_trace <call> n=<files> <phase>=<us> ...".
struct SdTrace {
  bool on;
  const char* call;
  size_t n;
  std::chrono::steady_clock::time_point t0, last;
  std::string line;
  SdTrace(bool on_, const char* call_, size_t n_) : on(on_), call(call_), n(n_) {
    if (on) t0 = last = std::chrono::steady_clock::now();
  }
  void note(const char* name, double v) {
    if (!on) return;
    char buf[64];
    snprintf(buf, sizeof buf, " %s=%.1f", name, v);
    line += buf;
  }
  void mark(const char* name) {
    if (!on) return;
    const auto t = std::chrono::steady_clock::now();
    char buf[64];
    snprintf(buf, sizeof buf, " %s=%.1f", name,
             std::chrono::duration<double, std::micro>(t - last).count());
    line += buf;
    last = t;
  }
  ~SdTrace() {
    if (!on) return;
    fprintf(stderr, "sd_cas_trace %s n=%zu%s total=%.1f\n", call, n, line.c_str(),
            std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
  }
};

// the NUMA node holding the page at p (get_mempolicy MPOL_F_NODE | MPOL_F_ADDR), -1 unknown
// (trace output only)
inline int sd_page_node(const void* p) {
  int node = -1;
  if (!p || syscall(SYS_get_mempolicy, &node, nullptr, 0UL, p, 3UL /* MPOL_F_NODE|MPOL_F_ADDR */) != 0)
    return -1;
  return node;
}

inline int sd_fail(sd_cas_ctx* c, int code, const char* fmt, ...) {
  if (c) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    c->err = buf;
  }
  return code;
}

#define HIP_TRY(ctx, expr)                                                                   \
  do {                                                                                       \
    hipError_t e_ = (expr);                                                                  \
    if (e_ != hipSuccess)                                                                    \
      return sd_fail((ctx), SD_CAS_EHIP, "%s failed: %s (%s:%d)", #expr, hipGetErrorString(e_), \
                     __FILE__, __LINE__);                                                    \
  } while (0)

// NULL = the HIP null (default) stream, exactly as in HIP itself: a caller on the
// default stream (torch's default) must be ordered with our kernels.
inline hipStream_t sd_pick(sd_cas_ctx*, void* s) { return (hipStream_t)s; }

// Order a use of the shared workspace (ws, d_scalar) on stream s after the previous use
// on any other stream; release records this use.  Calls on one stream need no event wait
// (stream order), so the single-stream pipelines pay one event record per call.
inline hipError_t sd_ws_acquire(sd_cas_ctx* c, hipStream_t s) {
  if (c->ws_pending && c->ws_stream != s) return hipStreamWaitEvent(s, c->ws_ev, 0);
  return hipSuccess;
}
inline hipError_t sd_ws_release(sd_cas_ctx* c, hipStream_t s) {
  c->ws_stream = s;
  c->ws_pending = true;
  return hipEventRecord(c->ws_ev, s);
}
inline size_t up16(size_t x) { return (x + 15) & ~(size_t)15; }
// packed whole-file contents start on 128-B lines: a K2 lane's line pair is one cache line
inline size_t up128(size_t x) { return (x + 127) & ~(size_t)127; }
inline size_t up256(size_t x) { return (x + 255) & ~(size_t)255; }

// Grow a device buffer (on the CURRENT device).  Growing synchronises the device: call
// outside hot loops / graph capture.
inline int sd_ensure(sd_cas_ctx* c, DevBuf& b, size_t bytes) {
  if (bytes <= b.bytes) return SD_CAS_OK;
  if (b.p) {
    HIP_TRY(c, hipDeviceSynchronize());
    HIP_TRY(c, hipFree(b.p));
    b.p = nullptr;
    b.bytes = 0;
  }
  size_t want = std::max(bytes, (size_t)1 << 20);
  if (hipMalloc(&b.p, want) != hipSuccess) {
    (void)hipGetLastError();
    return sd_fail(c, SD_CAS_ENOMEM, "hipMalloc(%zu) failed", want);
  }
  b.bytes = want;
  return SD_CAS_OK;
}

// The staging's host mapping.  SD_PINNED_MODE 0 = hipHostMallocDefault (the product), whose
// coherence follows HIP_HOST_COHERENT (unset = 0 = NON-coherent on ROCm); 1 = explicitly
// hipHostMallocNonCoherent; 2 = explicitly hipHostMallocCoherent.  Round 4's "coherent vs
// non-coherent" A/B compared modes 0 and 1 — with HIP_HOST_COHERENT unset both are the same
// non-coherent mapping, so it showed nothing; the three-arm A/B of round 5 with
// an explicit coherent arm is profiles/r05/ab_pinned_mode/ (DESIGN.md §2.2, f1).
#ifndef SD_PINNED_MODE
#define SD_PINNED_MODE 0
#endif
#define SD_PINNED_FLAGS                                                              \
  (SD_PINNED_MODE == 1 ? hipHostMallocNonCoherent                                    \
                       : SD_PINNED_MODE == 2 ? hipHostMallocCoherent : hipHostMallocDefault)

// K1 / K1L / K1+K1L by batch size (sd_hip_cas.cpp), shared with the host entry points
extern "C" hipError_t sd_dispatch_sampled(sd_cas_ctx* c, const uint8_t* content, uint64_t stride,
                                          const uint64_t* sizes, size_t n, uint64_t* keys,
                                          hipStream_t s);

inline int sd_ensure_pinned(sd_cas_ctx* c, size_t bytes) {
  if (bytes <= c->pinned_bytes) return SD_CAS_OK;
  if (c->pinned) {
    HIP_TRY(c, hipDeviceSynchronize());
    HIP_TRY(c, hipHostFree(c->pinned));
    c->pinned = nullptr;
    c->pinned_bytes = 0;
  }
  size_t want = std::max(bytes, (size_t)1 << 22);
  if (hipHostMalloc(&c->pinned, want, SD_PINNED_FLAGS) != hipSuccess) {
    (void)hipGetLastError();
    return sd_fail(c, SD_CAS_ENOMEM, "hipHostMalloc(%zu) failed", want);
  }
  c->pinned_bytes = want;
  return SD_CAS_OK;
}
