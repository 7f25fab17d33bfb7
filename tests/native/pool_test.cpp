// CPU test of the gather pool (spacedrive_amd/csrc/ctx_internal.h HostPool): many calls of
// run2/run with random worker counts, back to back and with pauses longer than the spin
// window (so workers park and are woken), each call's items all processed exactly once and
// the caller's own work done.  Exit 0 = ok.  Built by tests/test_host_pool.py.
#include <stdio.h>

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
  printf("pool ok\n");
  return 0;
}
