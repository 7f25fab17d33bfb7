// probe_pread.cpp — why does the validator's file path (sd_cas_file_checksums) read its
// 128 MB windows of tmpfs files at ~21 GB/s when 16 threads hashing the same files with
// 1 MiB reads reach 76 GB/s?  Reads 2,000 files of U(0.25, 4) MiB (written first) with T
// pthreads, files interleaved, in these forms:
//   scratch   1 MiB read()s into a per-thread buffer (cache-resident: what a CPU hasher does)
//   malloc    one pread per file into its slot of a 128 MB malloc'd window (as the pool does)
//   pinned    the same into hipHostMalloc'd memory (the library's staging)
//   pinned1m  1 MiB preads into the pinned window slots
//   pinned+dma the "pinned" form while the GPU copies another 128 MB pinned buffer to HBM
//             back to back (the file path double-buffers: window w is read while w-1 crosses)
//   product   sd_cas_file_checksums (include/sd_hip_cas.h) on the same files, from C
//   malloc1m / thp1m (round 6)  1 MiB preads into the malloc'd window / into a window of
//             transparent huge pages registered with hipHostRegister
// Build: hipcc --offload-arch=gfx950 -O2 -o tools/probe_pread tools/probe_pread.cpp -lpthread
#include <hip/hip_runtime.h>
#include <dlfcn.h>
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <pthread.h>
#include <unistd.h>

#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <vector>

static std::vector<std::string> paths;
static std::vector<uint64_t> sizes;

struct Job {
  int t, T, mode;
  char* win;
  const std::vector<uint64_t>* offs;
  size_t i0, i1;
};

static void* worker(void* p) {
  Job* j = (Job*)p;
  std::vector<char> scratch(1 << 20);
  for (size_t i = j->i0 + j->t; i < j->i1; i += j->T) {
    int fd = open(paths[i].c_str(), O_RDONLY);
    if (fd < 0) continue;
    if (j->mode == 0) {
      while (read(fd, scratch.data(), 1 << 20) == (1 << 20)) {
      }
    } else {
      char* dst = j->win + (*j->offs)[i - j->i0];
      uint64_t got = 0, n = sizes[i];
      while (got < n) {
        size_t want = j->mode == 3 ? std::min<uint64_t>(1 << 20, n - got) : n - got;
        ssize_t r = pread(fd, dst + got, want, (off_t)got);
        if (r <= 0) break;
        got += (uint64_t)r;
      }
    }
    close(fd);
  }
  return nullptr;
}

static double run(int mode, char* win, int T) {
  const uint64_t WIN = 128ull << 20;
  auto t0 = std::chrono::steady_clock::now();
  size_t i = 0;
  while (i < paths.size()) {
    std::vector<uint64_t> offs;
    uint64_t used = 0;
    size_t j = i;
    while (j < paths.size() && used + sizes[j] <= WIN) {
      offs.push_back(used);
      used += (sizes[j] + 127) / 128 * 128;
      j++;
    }
    std::vector<pthread_t> th(T);
    std::vector<Job> js(T);
    for (int t = 0; t < T; t++) {
      js[t] = {t, T, mode, win, &offs, i, j};
      pthread_create(&th[t], nullptr, worker, &js[t]);
    }
    for (int t = 0; t < T; t++) pthread_join(th[t], nullptr);
    i = j;
  }
  return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
}

int main(int argc, char** argv) {
  const int T = argc > 1 ? atoi(argv[1]) : 15;
  const char* root = "/dev/shm/sdcas_probe_pread";
  mkdir(root, 0755);
  std::mt19937_64 rng(6);
  std::vector<char> buf(4 << 20);
  for (auto& c : buf) c = (char)rng();
  uint64_t total = 0;
  for (int i = 0; i < 2000; i++) {
    uint64_t n = (1 << 18) + rng() % ((4 << 20) - (1 << 18));
    std::string p = std::string(root) + "/v" + std::to_string(i);
    FILE* f = fopen(p.c_str(), "wb");
    fwrite(buf.data(), 1, n, f);
    fclose(f);
    paths.push_back(p);
    sizes.push_back(n);
    total += n;
  }
  char* mwin = (char*)malloc((128u << 20) + (8u << 20));
  memset(mwin, 0, (128u << 20) + (8u << 20));
  char* pwin = nullptr;
  if (hipHostMalloc((void**)&pwin, (128u << 20) + (8u << 20), hipHostMallocDefault) != hipSuccess) return 1;
  // round 6: the same 1 MiB preads into a window of transparent huge pages (anonymous mmap +
  // MADV_HUGEPAGE, touched, then hipHostRegister'ed: DMA-able like the pinned staging) — does
  // the destination's page size bound the kernel's copy?
  const size_t tw = (128u << 20) + (8u << 20);
  char* thp = (char*)mmap(nullptr, tw, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
  if (thp == MAP_FAILED) return 1;
  (void)madvise(thp, tw, MADV_HUGEPAGE);
  memset(thp, 0, tw);
  const bool thp_reg = hipHostRegister(thp, tw, hipHostRegisterDefault) == hipSuccess;
  long anon_huge_kb = -1;
  if (FILE* f = fopen("/proc/self/smaps_rollup", "r")) {
    char line[256];
    while (fgets(line, sizeof line, f))
      if (!strncmp(line, "AnonHugePages:", 14)) anon_huge_kb = atol(line + 14);
    fclose(f);
  }
  printf("{\"thp_window\": true, \"registered\": %s, \"anon_huge_kb\": %ld}\n", thp_reg ? "true" : "false", anon_huge_kb);
  const char* names[] = {"scratch", "malloc", "pinned", "pinned1m", "malloc1m", "thp1m"};
  char* wins[] = {nullptr, mwin, pwin, pwin, mwin, thp};
  const int modes[] = {0, 1, 2, 3, 3, 3};
  for (int m = 0; m < 6; m++) {
    run(modes[m], wins[m], T);
    double best = 1e9;
    for (int r = 0; r < 3; r++) best = std::min(best, run(modes[m], wins[m], T));
    printf("{\"form\": \"%s\", \"threads\": %d, \"gb_per_s\": %.2f}\n", names[m], T, total / best / 1e9);
    fflush(stdout);
  }
  {  // pinned + concurrent H2D of a second pinned window
    char* pwin2 = nullptr;
    void* dbuf = nullptr;
    hipStream_t st;
    if (hipHostMalloc((void**)&pwin2, 128u << 20, hipHostMallocDefault) != hipSuccess ||
        hipMalloc(&dbuf, 128u << 20) != hipSuccess || hipStreamCreate(&st) != hipSuccess)
      return 1;
    memset(pwin2, 1, 128u << 20);
    for (int k = 0; k < 400; k++) (void)hipMemcpyAsync(dbuf, pwin2, 128u << 20, hipMemcpyHostToDevice, st);
    double best = 1e9;
    for (int r = 0; r < 3; r++) best = std::min(best, run(2, pwin, T));
    auto t0 = std::chrono::steady_clock::now();
    (void)hipStreamSynchronize(st);
    double tail = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    printf("{\"form\": \"pinned+dma\", \"threads\": %d, \"gb_per_s\": %.2f, \"dma_tail_s\": %.3f}\n",
           T, total / best / 1e9, tail);
    (void)hipStreamDestroy(st);
    (void)hipFree(dbuf);
    (void)hipHostFree(pwin2);
  }
  if (argc > 2) {  // the product's path: argv[2] = libsd_hip_cas.so
    void* h = dlopen(argv[2], RTLD_NOW | RTLD_LOCAL);
    typedef int (*create_fn)(int, void**);
    typedef int (*sums_fn)(void*, const char* const*, size_t, char*, int32_t*);
    create_fn create = h ? (create_fn)dlsym(h, "sd_cas_ctx_create") : nullptr;
    sums_fn sums = h ? (sums_fn)dlsym(h, "sd_cas_file_checksums") : nullptr;
    void* ctx = nullptr;
    if (!create || !sums || create(0, &ctx) != 0) return 2;
    std::vector<const char*> pp;
    for (auto& p : paths) pp.push_back(p.c_str());
    std::vector<char> hex(65 * paths.size());
    std::vector<int32_t> st(paths.size());
    sums(ctx, pp.data(), pp.size(), hex.data(), st.data());
    double best = 1e9;
    for (int r = 0; r < 3; r++) {
      auto t0 = std::chrono::steady_clock::now();
      sums(ctx, pp.data(), pp.size(), hex.data(), st.data());
      best = std::min(best, std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count());
    }
    printf("{\"form\": \"product\", \"gb_per_s\": %.2f}\n", total / best / 1e9);
  }
  for (auto& p : paths) unlink(p.c_str());
  rmdir(root);
  (void)hipHostFree(pwin);
  free(mwin);
  return 0;
}
