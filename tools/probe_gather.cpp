// probe_gather.cpp (round 6) — does config 1's gather (sd_cas_generate_cas_keys_from_paths,
// host_paths.cpp) pay for the destination it writes?  The product's readers write each file's
// cas.rs content (cas.rs:23-62: header + sample 0 as one pread, samples 1-3, fstat, footer;
// whole files <= 100 KiB read whole after an fstat) into its slot of one pinned window of
// ~830 files (~33 MB): every byte lands in DRAM before the DMA reads it.  This probe reads
// config 1's file mix (10,000 tmpfs files, log-uniform 1 KiB..10 MiB, tools/bench_configs.py)
// with T pthreads in these forms:
//   window    each file into its slot of a 36 MB pinned window, windows of 830 files (product)
//   malloc    the same into a malloc'd window
//   ring      each thread into its own 2 MiB pinned ring (reused: stays cache-resident)
//   ring+h2d  the ring form, each filled 512 KiB quarter of a ring copied to HBM with
//             hipMemcpyAsync on one of 2 streams before the thread reuses it (event-gated)
//   unshared  the window form, each reader first calling unshare(CLONE_FILES): a private
//             descriptor table, so open/close stop sharing the process's table lock
//   openat    the unshared form, each reader opening the files by name relative to its own
//             descriptor of their directory (openat): no absolute-path walk from "/"
// argv: T files [sweep] — with "sweep", the window, unshared and openat forms at T = 1..16.
// Build: hipcc --offload-arch=gfx950 -O2 -o tools/probe_gather tools/probe_gather.cpp -lpthread
#include <hip/hip_runtime.h>
#include <fcntl.h>
#include <sched.h>
#include <pthread.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <mutex>
#include <random>
#include <string>
#include <vector>

static std::vector<std::string> paths;
static std::vector<uint64_t> sizes;
static constexpr uint64_t MIN_FILE = 100 * 1024, CONTENT = 57344, RING = 2u << 20, QUARTER = RING / 4;

// one file's cas.rs reads into dst; returns bytes written
static std::vector<std::string> names;  // the files' names in their directory
static uint64_t read_item(size_t i, char* dst, int dirfd = -1) {
  const int fd = dirfd >= 0 ? openat(dirfd, names[i].c_str(), O_RDONLY | O_CLOEXEC)
                            : open(paths[i].c_str(), O_RDONLY | O_CLOEXEC);
  if (fd < 0) return 0;
  struct stat st;
  uint64_t offs[5], lns[5];
  int parts;
  if (sizes[i] <= MIN_FILE) {
    if (fstat(fd, &st) != 0) { close(fd); return 0; }
    offs[0] = 0; lns[0] = sizes[i]; parts = 1;
  } else {
    const uint64_t jump = (sizes[i] - 16384) / 4;
    offs[0] = 0; lns[0] = 18432;
    for (int k = 1; k < 4; k++) { offs[k] = 8192 + k * jump; lns[k] = 10240; }
    lns[4] = 8192; parts = 5;
  }
  uint64_t w = 0;
  for (int k = 0; k < parts; k++) {
    if (k == 4) {
      if (fstat(fd, &st) != 0) break;
      offs[4] = (uint64_t)st.st_size - 8192;
    }
    if (pread(fd, dst + w, lns[k], (off_t)offs[k]) != (ssize_t)lns[k]) break;
    w += lns[k];
  }
  close(fd);
  return w;
}

struct Shared {
  int mode, T;
  char* win;
  const std::vector<uint64_t>* offs;
  size_t i0, i1;
  std::atomic<size_t> next;
  char* rings;     // T rings
  char* dev;       // T rings on the device
  hipStream_t st[2];
  std::mutex mu;
  const char* dir;
};
struct Arg { Shared* s; int t; };

static void* worker(void* p) {
  Arg* a = (Arg*)p;
  Shared* s = a->s;
  if ((s->mode == 4 || s->mode == 5) && unshare(CLONE_FILES) != 0) perror("unshare");
  const int dirfd = s->mode == 5 ? open(s->dir, O_RDONLY | O_DIRECTORY | O_CLOEXEC) : -1;
  char* ring = s->rings ? s->rings + (size_t)a->t * RING : nullptr;
  hipEvent_t ev[4] = {};
  if (s->mode == 3)
    for (auto& e : ev) (void)hipEventCreateWithFlags(&e, hipEventDisableTiming);
  uint64_t pos = 0;  // ring fill position (bytes since start)
  for (size_t i; (i = s->next.fetch_add(1)) < s->i1;) {
    if (s->mode <= 1 || s->mode >= 4) {
      read_item(i, s->win + (*s->offs)[i - s->i0], dirfd);
      continue;
    }
    // ring: the file's content at the fill position (wrapping to the ring start when the
    // item would cross the end); with h2d, each quarter crossed is sent, and a quarter is
    // reused only after its copy's event
    const uint64_t need = sizes[i] <= MIN_FILE ? sizes[i] : CONTENT;
    uint64_t at = pos % RING;
    if (at + need > RING) { pos += RING - at; at = 0; }
    if (s->mode == 3) {
      const int q0 = (int)(at / QUARTER), q1 = (int)((at + need - 1) / QUARTER);
      for (int q = q0; q <= q1; q++) (void)hipEventSynchronize(ev[q]);
    }
    const uint64_t before = pos;
    read_item(i, ring + at);
    pos += (need + 127) / 128 * 128;
    if (s->mode == 3) {
      // quarters completed by this item
      for (uint64_t q = before / QUARTER; q < pos / QUARTER; q++) {
        const int qi = (int)(q % 4);
        hipStream_t st = s->st[(a->t + q) & 1];
        (void)hipMemcpyAsync(s->dev + (size_t)a->t * RING + qi * QUARTER, ring + qi * QUARTER, QUARTER,
                             hipMemcpyHostToDevice, st);
        (void)hipEventRecord(ev[qi], st);
      }
    }
  }
  if (s->mode == 3)
    for (auto& e : ev) { (void)hipEventSynchronize(e); (void)hipEventDestroy(e); }
  if (dirfd >= 0) close(dirfd);
  return nullptr;
}

static double run(int mode, Shared& s, char* win) {
  const uint64_t WIN = 36ull << 20;
  auto t0 = std::chrono::steady_clock::now();
  size_t i = 0;
  while (i < paths.size()) {
    std::vector<uint64_t> offs;
    uint64_t used = 0;
    size_t j = i;
    // the product's windows: ~830 files (total / 12 staged bytes)
    while (j < paths.size() && j - i < 830 && used + CONTENT <= WIN) {
      offs.push_back(used);
      used += ((sizes[j] <= MIN_FILE ? sizes[j] : CONTENT) + 127) / 128 * 128;
      j++;
    }
    s.mode = mode; s.win = win; s.offs = &offs; s.i0 = i; s.i1 = j; s.next.store(i);
    std::vector<pthread_t> th(s.T);
    std::vector<Arg> as(s.T);
    for (int t = 0; t < s.T; t++) {
      as[t] = {&s, t};
      pthread_create(&th[t], nullptr, worker, &as[t]);
    }
    for (int t = 0; t < s.T; t++) pthread_join(th[t], nullptr);
    i = j;
  }
  return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
}

int main(int argc, char** argv) {
  const int T = argc > 1 ? atoi(argv[1]) : 16;
  const int N = argc > 2 ? atoi(argv[2]) : 10000;
  const char* root = "/dev/shm/sdcas_probe_gather";
  mkdir(root, 0755);
  std::mt19937_64 rng(1);
  std::uniform_real_distribution<double> U(std::log(1024.0), std::log(10.0 * 1024 * 1024));
  std::vector<char> buf(10u << 20);
  for (auto& c : buf) c = (char)rng();
  uint64_t staged = 0;
  for (int i = 0; i < N; i++) {
    const uint64_t n = (uint64_t)std::exp(U(rng));
    std::string p = std::string(root) + "/f" + std::to_string(i);
    FILE* f = fopen(p.c_str(), "wb");
    if (!f || fwrite(buf.data(), 1, n, f) != n) return 1;
    fclose(f);
    paths.push_back(p);
    names.push_back("f" + std::to_string(i));
    sizes.push_back(n);
    staged += n <= MIN_FILE ? n : CONTENT;
  }
  char* mwin = (char*)malloc(40u << 20);
  char* pwin = nullptr;
  Shared s;
  s.T = T;
  s.dir = root;
  if (hipHostMalloc((void**)&pwin, 40u << 20, hipHostMallocDefault) != hipSuccess ||
      hipHostMalloc((void**)&s.rings, (size_t)T * RING, hipHostMallocDefault) != hipSuccess ||
      hipMalloc((void**)&s.dev, (size_t)T * RING) != hipSuccess ||
      hipStreamCreateWithFlags(&s.st[0], hipStreamNonBlocking) != hipSuccess ||
      hipStreamCreateWithFlags(&s.st[1], hipStreamNonBlocking) != hipSuccess)
    return 2;
  std::fill(mwin, mwin + (40u << 20), 0);
  std::fill(pwin, pwin + (40u << 20), 0);
  std::fill(s.rings, s.rings + (size_t)T * RING, 0);
  const char* forms[] = {"window", "malloc", "ring", "ring+h2d", "unshared", "openat"};
  char* wins[] = {pwin, mwin, nullptr, nullptr, pwin, pwin};
  const bool sweep = argc > 3 && std::string(argv[3]) == "sweep";
  std::vector<std::pair<int, int>> plan;  // (threads, mode)
  for (int round = 0; round < 2; round++)
    if (sweep)
      for (int t : {1, 2, 4, 8, 16})
        for (int m : {0, 4, 5}) plan.push_back({t, m});
    else
      for (int m = 0; m < 6; m++) plan.push_back({T, m});
  for (size_t pi = 0; pi < plan.size(); pi++) {
      const int m = plan[pi].second, round = (int)(pi * 2 / plan.size());
      s.T = plan[pi].first;
      run(m, s, wins[m]);
      std::vector<double> ts;
      for (int r = 0; r < 5; r++) ts.push_back(run(m, s, wins[m]));
      std::sort(ts.begin(), ts.end());
      printf("{\"form\": \"%s\", \"round\": %d, \"threads\": %d, \"files\": %d, \"staged_mb\": %.1f, "
             "\"median_s\": %.5f, \"files_per_s\": %.0f, \"gb_per_s\": %.2f}\n",
             forms[m], round, s.T, N, staged / 1e6, ts[2], N / ts[2], staged / ts[2] / 1e9);
      fflush(stdout);
    }
  for (auto& p : paths) unlink(p.c_str());
  rmdir(root);
  return 0;
}
