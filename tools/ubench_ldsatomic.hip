// ubench_ldsatomic.hip — gfx950 LDS atomic throughput at random slots (the grouping's
// K5h insert: 64-bit CAS + 32-bit min into a 4,096-slot table), 3 workgroups of 512 lanes
// per CU like sd_bucket_min.  Prints lane-ops per cycle per CU for each op.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/ubench_ldsatomic tools/ubench_ldsatomic.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)
constexpr int TBL = 4096, ITERS = 256;

__device__ __forceinline__ uint32_t hsh(uint32_t x) { x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; return x ^ (x >> 16); }

template <int MODE>
__global__ void __launch_bounds__(512) k(uint32_t* out, uint32_t seed) {
  __shared__ uint64_t tk[TBL];
  __shared__ uint32_t tv[TBL];
  for (int i = threadIdx.x; i < TBL; i += 512) { tk[i] = 0; tv[i] = 0xFFFFFFFFu; }
  __syncthreads();
  uint32_t acc = 0, st = hsh(threadIdx.x ^ seed ^ (blockIdx.x << 10));
#pragma unroll 1
  for (int it = 0; it < ITERS; ++it) {
    st = hsh(st + it);
    const uint32_t s = st & (TBL - 1);
    if (MODE == 0) {  // CAS 64
      acc += (uint32_t)atomicCAS((unsigned long long*)&tk[s], 0ull, (unsigned long long)st | 1ull);
    } else if (MODE == 1) {  // min 32
      acc += atomicMin(&tv[s], st);
    } else if (MODE == 2) {  // CAS + min (the insert)
      acc += (uint32_t)atomicCAS((unsigned long long*)&tk[s], 0ull, (unsigned long long)st | 1ull);
      atomicMin(&tv[s], st);
    } else if (MODE == 3) {  // plain 64-bit read
      acc += (uint32_t)tk[s];
    } else {  // min without return
      atomicMin(&tv[s], st);
    }
  }
  out[blockIdx.x * 512 + threadIdx.x] = acc;
}

int main() {
  hipDeviceProp_t p;
  CHECK(hipGetDeviceProperties(&p, 0));
  const int cus = p.multiProcessorCount, blocks = cus * 3 * 8;
  uint32_t* out;
  CHECK(hipMalloc(&out, (size_t)blocks * 512 * 4));
  hipEvent_t a, b;
  (void)hipEventCreate(&a); (void)hipEventCreate(&b);
  const char* names[] = {"CAS64 rtn", "min32 rtn", "CAS64+min32", "read64", "min32 no-rtn"};
  void (*ks[])(uint32_t*, uint32_t) = {k<0>, k<1>, k<2>, k<3>, k<4>};
  for (int m = 0; m < 5; ++m) {
    hipLaunchKernelGGL(ks[m], dim3(blocks), dim3(512), 0, 0, out, 1u);
    CHECK(hipDeviceSynchronize());
    (void)hipEventRecord(a, 0);
    hipLaunchKernelGGL(ks[m], dim3(blocks), dim3(512), 0, 0, out, 2u);
    (void)hipEventRecord(b, 0);
    CHECK(hipEventSynchronize(b));
    float ms;
    (void)hipEventElapsedTime(&ms, a, b);
    const double ops = (double)blocks * 512 * ITERS * (m == 2 ? 2 : 1);
    printf("%-14s %8.3f ms  %.2f lane-ops/cycle/CU at 2.4 GHz  (%.1f G lane-ops/s)\n", names[m], ms,
           ops / cus / (ms * 1e-3 * 2.4e9), ops / (ms * 1e-3) / 1e9);
  }
  return 0;
}
