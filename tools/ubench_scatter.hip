// ubench_scatter.hip — cost of scattered stores on MI355X at the grouping's sizes: a
// coalesced copy, fully random 4-B and 8-B scatters (the rep write of K5h, the single-level
// partition), and scatters whose destinations come in contiguous runs of R elements (what a
// partition with n/R keys per bucket per block produces).
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/ubench_scatter tools/ubench_scatter.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include <algorithm>
#include <numeric>
#include <random>
#include <vector>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

__global__ void copy64(const uint64_t* __restrict__ in, uint64_t* __restrict__ out, uint64_t n) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    out[i] = in[i];
}
__global__ void scatter32(const uint32_t* __restrict__ perm, uint32_t* __restrict__ out, uint64_t n) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    out[perm[i]] = (uint32_t)i;
}
__global__ void scatter64(const uint32_t* __restrict__ perm, const uint64_t* __restrict__ in,
                          uint64_t* __restrict__ out, uint64_t n) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    out[perm[i]] = in[i];
}
__global__ void gather32(const uint32_t* __restrict__ perm, const uint32_t* __restrict__ in,
                         uint32_t* __restrict__ out, uint64_t n) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    out[i] = in[perm[i]];
}

int main() {
  const uint64_t n = 12500000;
  std::vector<uint32_t> h(n);
  std::mt19937_64 rng(1);
  uint32_t *perm, *o32, *i32;
  uint64_t *i64, *o64;
  CHECK(hipMalloc(&perm, n * 4));
  CHECK(hipMalloc(&o32, n * 4));
  CHECK(hipMalloc(&i32, n * 4));
  CHECK(hipMalloc(&i64, n * 8));
  CHECK(hipMalloc(&o64, n * 8));
  CHECK(hipMemset(i64, 1, n * 8));
  CHECK(hipMemset(i32, 1, n * 4));
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  auto timeit = [&](auto launch) {
    launch();
    (void)hipDeviceSynchronize();
    float best = 1e9;
    for (int r = 0; r < 5; ++r) {
      (void)hipEventRecord(a, 0);
      launch();
      (void)hipEventRecord(b, 0);
      (void)hipEventSynchronize(b);
      float ms;
      (void)hipEventElapsedTime(&ms, a, b);
      best = std::min(best, ms);
    }
    return best;
  };
  const dim3 g(4096), t(256);
  float ms = timeit([&] { copy64<<<g, t>>>(i64, o64, n); });
  printf("copy 8 B/elem            %8.1f us  %6.0f GB/s (16 B/elem moved)\n", ms * 1e3, 16.0 * n / ms / 1e6);
  for (uint32_t run : {1u, 4u, 16u, 64u, 256u, 4096u}) {
    // destinations: runs of `run` consecutive slots, runs in random order
    const uint64_t nr = (n + run - 1) / run;
    std::vector<uint32_t> order(nr);
    std::iota(order.begin(), order.end(), 0u);
    std::shuffle(order.begin(), order.end(), rng);
    uint64_t k = 0;
    for (uint64_t r = 0; r < nr && k < n; ++r)
      for (uint32_t j = 0; j < run && k < n; ++j) {
        const uint64_t d = (uint64_t)order[r] * run + j;
        h[k++] = (uint32_t)(d < n ? d : (d % n));
      }
    // make it a permutation again for the tail run
    if (n % run) {
      std::vector<char> seen(n, 0);
      std::vector<uint32_t> free_;
      for (uint64_t i = 0; i < n; ++i) seen[h[i]] = 1;
      for (uint64_t i = 0; i < n; ++i) if (!seen[i]) free_.push_back((uint32_t)i);
      std::vector<char> used(n, 0);
      size_t f = 0;
      for (uint64_t i = 0; i < n; ++i) { if (used[h[i]]) h[i] = free_[f++]; used[h[i]] = 1; }
    }
    CHECK(hipMemcpy(perm, h.data(), n * 4, hipMemcpyHostToDevice));
    float s32 = timeit([&] { scatter32<<<g, t>>>(perm, o32, n); });
    float s64 = timeit([&] { scatter64<<<g, t>>>(perm, i64, o64, n); });
    float g32 = timeit([&] { gather32<<<g, t>>>(perm, i32, o32, n); });
    printf("run %5u: scatter 4 B %7.1f us (%5.0f GB/s of 8 B/elem)  scatter 8 B %7.1f us (%5.0f GB/s of 20 B/elem)  gather 4 B %7.1f us\n",
           run, s32 * 1e3, 8.0 * n / s32 / 1e6, s64 * 1e3, 20.0 * n / s64 / 1e6, g32 * 1e3);
  }
  return 0;
}
