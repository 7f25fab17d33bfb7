// CPU test of the gather pool (spacedrive_amd/csrc/ctx_internal.h HostPool): many calls of
// run2/run with random worker counts, back to back and with pauses longer than the spin
// window (so workers park and are woken), each call's items all processed exactly once and
// the caller's own work done.  Round 6: the private descriptor tables (set_private_fds) — the
// pool's threads see none of the caller's descriptors (a pipe here), open and read files of
// their own, and the caller's pipe reaches EOF when the caller closes its write end; shared
// mode sees the pipe.  Exit 0 = ok.  Built by tests/test_host_pool.py.
#include <fcntl.h>
#include <poll.h>
#include <stdio.h>
#include <string.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <random>
#include <thread>
#include <vector>

#include "ctx_internal.h"

int main() {
  HostPool pool;
  std::mt19937 rng(7);
  for (int call = 0; call < 4000; ++call) {
    const unsigned workers = 1 + rng() % 15;
    const size_t items = rng() % 300;
    std::vector<std::atomic<int>> hit(items);
    for (auto& h : hit) h.store(0);
    std::atomic<size_t> next{0};
    std::atomic<int> callers{0};
    auto fn = [&]() {
      for (size_t t; (t = next.fetch_add(1)) < items;) hit[t].fetch_add(1);
    };
    auto caller = [&]() { callers.fetch_add(1); fn(); };
    if (call % 3 == 0)
      pool.run(workers + 1, fn);
    else
      pool.run2(workers, fn, caller);
    for (size_t t = 0; t < items; ++t)
      if (hit[t].load() != 1) { printf("call %d: item %zu hit %d times\n", call, t, hit[t].load()); return 1; }
    if (call % 3 != 0 && callers.load() != 1) { printf("call %d: caller ran %d times\n", call, callers.load()); return 1; }
    if (call % 97 == 0) std::this_thread::sleep_for(std::chrono::microseconds(300 + rng() % 2000));
  }
  for (int mode = 1; mode >= 0; --mode) {
    int pfd[2];
    if (pipe(pfd) != 0) return 1;
    char tmpl[] = "/tmp/sd_pool_fdXXXXXX";
    const int tf = mkstemp(tmpl);
    if (tf < 0 || write(tf, "hello", 5) != 5) return 1;
    close(tf);
    std::atomic<int> sees_pipe{0}, read_ok{0};
    const unsigned W = 4;
    {
      HostPool p2;
      p2.set_private_fds(mode == 1);
      p2.run2(W, [&]() {
        if (fcntl(pfd[1], F_GETFD) != -1) sees_pipe.fetch_add(1);
        const int fd = open(tmpl, O_RDONLY | O_CLOEXEC);
        char b[8];
        if (fd >= 0 && pread(fd, b, 5, 0) == 5 && !memcmp(b, "hello", 5)) read_ok.fetch_add(1);
        if (fd >= 0) close(fd);
      }, []() {});
      const int want_private = mode == 1 ? (int)W : 0, want_sees = mode == 1 ? 0 : (int)W;
      if (p2.private_threads() != want_private || sees_pipe.load() != want_sees || read_ok.load() != (int)W) {
        printf("mode %d: private threads %d, threads seeing the pipe %d, reads ok %d\n", mode,
               p2.private_threads(), sees_pipe.load(), read_ok.load());
        return 1;
      }
      // the pool still lives: the pipe must reach EOF once the caller closes its write end
      close(pfd[1]);
      pollfd q{pfd[0], POLLIN, 0};
      char c;
      if (poll(&q, 1, 2000) != 1 || read(pfd[0], &c, 1) != 0) {
        printf("mode %d: the pipe did not reach EOF\n", mode);
        return 1;
      }
    }
    close(pfd[0]);
    unlink(tmpl);
  }
  printf("pool ok\n");
  return 0;
}
