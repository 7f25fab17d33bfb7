// probe_mmap_reg.cpp — can the validator's file path skip the host-side copy?  Today each
// file is pread into pinned staging (host memory: read the page cache + write the staging)
// and then DMA'd to HBM (read the staging again).  This probe maps each tmpfs file, registers
// the mapping with hipHostRegister and DMAs the page-cache pages straight to HBM (one host
// memory read per byte).  2,000 files of U(0.25, 4) MiB (written first, as probe_pread.cpp).
// Forms (best of 3, one JSON line each):
//   reg_only   T threads: open + mmap + hipHostRegister + hipHostUnregister + munmap per file
//   reg_dma    windows of 128 MiB: T threads map + register the window's files, this thread
//              DMAs each file to its slot as it is registered (one stream), then unregisters
//   the copied bytes of every file are checked against the file once (memcmp after D2H)
// Build: hipcc --offload-arch=gfx950 -O2 -o tools/probe_mmap_reg tools/probe_mmap_reg.cpp -lpthread
#include <hip/hip_runtime.h>
#include <fcntl.h>
#include <pthread.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <thread>
#include <vector>

static std::vector<std::string> paths;
static std::vector<uint64_t> sizes;

struct Mapped {
  void* p = nullptr;
  uint64_t len = 0;  // mapped bytes (page multiple)
  int err = 0;
};

static int map_register(size_t i, Mapped& m) {
  int fd = open(paths[i].c_str(), O_RDONLY | O_CLOEXEC);
  if (fd < 0) return m.err = errno;
  struct stat st;
  if (fstat(fd, &st) != 0) { m.err = errno; close(fd); return m.err; }
  m.len = ((uint64_t)st.st_size + 4095) / 4096 * 4096;
  m.p = mmap(nullptr, m.len, PROT_READ, MAP_SHARED | MAP_POPULATE, fd, 0);
  close(fd);
  if (m.p == MAP_FAILED) { m.p = nullptr; return m.err = errno; }
  hipError_t e = hipHostRegister(m.p, m.len, hipHostRegisterReadOnly);
  if (e != hipSuccess) {
    fprintf(stderr, "hipHostRegister: %s\n", hipGetErrorString(e));
    munmap(m.p, m.len);
    m.p = nullptr;
    return m.err = 1000;
  }
  return 0;
}

static void unmap(Mapped& m) {
  if (!m.p) return;
  (void)hipHostUnregister(m.p);
  munmap(m.p, m.len);
  m.p = nullptr;
}

static double reg_only(int T) {
  std::atomic<size_t> next{0};
  std::atomic<int> bad{0};
  auto t0 = std::chrono::steady_clock::now();
  std::vector<std::thread> th;
  for (int t = 0; t < T; t++)
    th.emplace_back([&]() {
      for (size_t i; (i = next.fetch_add(1)) < paths.size();) {
        Mapped m;
        if (map_register(i, m)) bad++;
        unmap(m);
      }
    });
  for (auto& x : th) x.join();
  if (bad) fprintf(stderr, "reg_only: %d failures\n", bad.load());
  return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
}

static double reg_dma(int T, char* dev, hipStream_t s, bool check) {
  const uint64_t WIN = 128ull << 20;
  auto t0 = std::chrono::steady_clock::now();
  size_t i = 0;
  std::vector<Mapped> maps(paths.size());
  std::vector<uint64_t> doff(paths.size());
  while (i < paths.size()) {
    size_t j = i;
    uint64_t used = 0;
    while (j < paths.size() && used + sizes[j] + 4096 <= WIN) { doff[j] = used; used += (sizes[j] + 4095) / 4096 * 4096; j++; }
    std::atomic<size_t> next{i};
    std::vector<std::atomic<uint8_t>> fin(j - i);
    for (auto& f : fin) f.store(0);
    std::vector<std::thread> th;
    for (int t = 0; t < T; t++)
      th.emplace_back([&]() {
        for (size_t k; (k = next.fetch_add(1)) < j;) {
          map_register(k, maps[k]);
          fin[k - i].store(1, std::memory_order_release);
        }
      });
    for (size_t k = i; k < j; k++) {  // DMA each file as soon as it is registered
      while (!fin[k - i].load(std::memory_order_acquire)) std::this_thread::yield();
      if (maps[k].p) (void)hipMemcpyAsync(dev + doff[k], maps[k].p, (sizes[k] + 15) / 16 * 16, hipMemcpyHostToDevice, s);
    }
    for (auto& x : th) x.join();
    (void)hipStreamSynchronize(s);
    if (check) {
      std::vector<char> buf;
      for (size_t k = i; k < j; k++) {
        buf.resize(sizes[k]);
        (void)hipMemcpy(buf.data(), dev + doff[k], sizes[k], hipMemcpyDeviceToHost);
        if (!maps[k].p || memcmp(buf.data(), maps[k].p, sizes[k]) != 0) { fprintf(stderr, "mismatch file %zu\n", k); exit(3); }
      }
    }
    for (size_t k = i; k < j; k++) unmap(maps[k]);
    i = j;
  }
  return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
}

int main(int argc, char** argv) {
  const int T = argc > 1 ? atoi(argv[1]) : 15;
  const char* root = "/dev/shm/sdcas_probe_mmap";
  mkdir(root, 0755);
  std::mt19937_64 rng(6);
  std::vector<char> buf(4 << 20);
  for (auto& c : buf) c = (char)rng();
  uint64_t total = 0;
  for (int i = 0; i < 2000; i++) {
    uint64_t n = (1 << 18) + rng() % ((4 << 20) - (1 << 18));
    std::string p = std::string(root) + "/v" + std::to_string(i);
    FILE* f = fopen(p.c_str(), "wb");
    fwrite(buf.data() + (i % 64), 1, n, f);
    fclose(f);
    paths.push_back(p);
    sizes.push_back(n);
    total += n;
  }
  char* dev = nullptr;
  hipStream_t s;
  if (hipMalloc(&dev, 136u << 20) != hipSuccess || hipStreamCreate(&s) != hipSuccess) return 1;
  {
    double best = 1e9;
    for (int r = 0; r < 3; r++) best = std::min(best, reg_only(T));
    printf("{\"form\": \"reg_only\", \"threads\": %d, \"files_per_s\": %.0f, \"gb_per_s\": %.2f}\n", T,
           paths.size() / best, total / best / 1e9);
    fflush(stdout);
  }
  reg_dma(T, dev, s, true);  // warm + byte check
  for (int TT : {T, 8, 4}) {
    double best = 1e9;
    for (int r = 0; r < 3; r++) best = std::min(best, reg_dma(TT, dev, s, false));
    printf("{\"form\": \"reg_dma\", \"threads\": %d, \"gb_per_s\": %.2f, \"checked\": true}\n", TT, total / best / 1e9);
    fflush(stdout);
  }
  for (auto& p : paths) unlink(p.c_str());
  rmdir(root);
  return 0;
}
