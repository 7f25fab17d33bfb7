// ubench_gridsync.hip — what does a grid-wide barrier cost on MI355X, against the gap
// between two dependent kernel launches on one stream?  (Prices a persistent single-launch
// grouping against the current 7-8 launch chain.)
//   a. cooperative launch + cooperative_groups grid.sync()
//   b. hand-written barrier: one global atomic arrive per workgroup + spin on a generation
//      word (vector atomics / loads only)
//   c. back-to-back empty launches, and launches that each touch 1 MB
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/ubench_gridsync tools/ubench_gridsync.hip
#include <hip/hip_cooperative_groups.h>
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

namespace cg = cooperative_groups;

#define CHECK(x)                                                                  \
  do {                                                                            \
    hipError_t e = (x);                                                           \
    if (e != hipSuccess) {                                                        \
      fprintf(stderr, "%s: %s (%s:%d)\n", #x, hipGetErrorString(e), __FILE__, __LINE__); \
      exit(1);                                                                    \
    }                                                                             \
  } while (0)

__global__ void k_coop(int iters, unsigned* sink) {
  cg::grid_group g = cg::this_grid();
  unsigned acc = 0;
  for (int i = 0; i < iters; ++i) {
    acc += threadIdx.x ^ i;
    g.sync();
  }
  if (acc == 0xFFFFFFFFu) sink[0] = acc;
}

// arrive: one atomicAdd per workgroup; the last arriver bumps the generation
__device__ __forceinline__ void grid_barrier(unsigned* count, unsigned* gen, unsigned nblocks) {
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned g0 = __hip_atomic_load(gen, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned arrived = atomicAdd(count, 1u) + 1u;
    if (arrived == nblocks) {
      __hip_atomic_store(count, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_fetch_add(gen, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      while (__hip_atomic_load(gen, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) == g0)
        __builtin_amdgcn_s_sleep(1);
    }
  }
  __syncthreads();
}

__global__ void k_custom(int iters, unsigned* count, unsigned* gen, unsigned* sink) {
  unsigned acc = 0;
  for (int i = 0; i < iters; ++i) {
    acc += threadIdx.x ^ i;
    grid_barrier(count, gen, gridDim.x);
  }
  if (acc == 0xFFFFFFFFu) sink[0] = acc;
}

__global__ void k_empty(unsigned* sink) {
  if (threadIdx.x == 0xFFFFFFFFu) sink[0] = 1;
}

__global__ void k_touch(const uint4* in, uint4* out, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    out[i] = in[i];
}

int main() {
  hipDeviceProp_t p;
  CHECK(hipGetDeviceProperties(&p, 0));
  const int cus = p.multiProcessorCount;
  unsigned *sink, *count, *gen;
  CHECK(hipMalloc(&sink, 64));
  CHECK(hipMalloc(&count, 64));
  CHECK(hipMalloc(&gen, 64));
  CHECK(hipMemset(count, 0, 64));
  CHECK(hipMemset(gen, 0, 64));
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  float ms;
  const int iters = 2000;
  for (int threads : {256, 1024}) {
    int per_cu = 0;
    CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_coop, threads, 0));
    const int blocks = cus * (per_cu < 1 ? 1 : (per_cu > 2 ? 2 : per_cu));
    void* args[] = {(void*)&iters, (void*)&sink};
    CHECK(hipLaunchCooperativeKernel((void*)k_coop, dim3(blocks), dim3(threads), args, 0, 0));
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventRecord(a));
    CHECK(hipLaunchCooperativeKernel((void*)k_coop, dim3(blocks), dim3(threads), args, 0, 0));
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    CHECK(hipEventElapsedTime(&ms, a, b));
    printf("{\"variant\": \"coop_grid_sync\", \"blocks\": %d, \"threads\": %d, \"us_per_barrier\": %.3f}\n",
           blocks, threads, ms * 1e3 / iters);
    const int cblocks = cus;  // one workgroup per CU: always co-resident
    k_custom<<<cblocks, threads>>>(10, count, gen, sink);
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventRecord(a));
    k_custom<<<cblocks, threads>>>(iters, count, gen, sink);
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    CHECK(hipEventElapsedTime(&ms, a, b));
    printf("{\"variant\": \"custom_barrier\", \"blocks\": %d, \"threads\": %d, \"us_per_barrier\": %.3f}\n",
           cblocks, threads, ms * 1e3 / iters);
  }
  // back-to-back launches on one stream
  for (int blocks : {256, 1024}) {
    for (int i = 0; i < 10; ++i) k_empty<<<blocks, 256>>>(sink);
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventRecord(a));
    for (int i = 0; i < iters; ++i) k_empty<<<blocks, 256>>>(sink);
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    CHECK(hipEventElapsedTime(&ms, a, b));
    printf("{\"variant\": \"empty_launch\", \"blocks\": %d, \"us_per_launch\": %.3f}\n", blocks,
           ms * 1e3 / iters);
  }
  const size_t bytes = 1 << 20;
  uint4 *x, *y;
  CHECK(hipMalloc(&x, bytes));
  CHECK(hipMalloc(&y, bytes));
  for (int i = 0; i < 10; ++i) k_touch<<<256, 256>>>(x, y, bytes / 16);
  CHECK(hipDeviceSynchronize());
  CHECK(hipEventRecord(a));
  for (int i = 0; i < iters; ++i) k_touch<<<256, 256>>>(x, y, bytes / 16);
  CHECK(hipEventRecord(b));
  CHECK(hipEventSynchronize(b));
  CHECK(hipEventElapsedTime(&ms, a, b));
  printf("{\"variant\": \"copy_1MiB_launch\", \"blocks\": 256, \"us_per_launch\": %.3f}\n", ms * 1e3 / iters);
  return 0;
}
