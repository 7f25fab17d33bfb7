// ubench_k1.hip — where K1 (sampled lane-per-file kernel) loses against the compute-only
// compression loop: the same lane code with its loads aimed at HBM (real layout), at an
// L2-resident window, or broadcast (every lane the same file), plus the compute-only loop,
// each with the shader clock measured inside the kernel (s_memtime / s_memrealtime).
// Build: hipcc --offload-arch=gfx950 -O3 -I spacedrive_amd/csrc -I include -o tools/ubench_k1 tools/ubench_k1.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include "../spacedrive_amd/csrc/cas_hash.hip"

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

// mode 0: real (file f), 1: window of 32 files (L2), 2: broadcast (file 0 for every lane),
// 4: real with non-temporal loads, 5: LINE-tiled layout (64-file tiles, 128-B lines
// interleaved), 6: QUAD-tiled layout (16-B quads interleaved: every load coalesced)
template <int MODE>
__global__ void __launch_bounds__(256) k1_variant(const uint8_t* __restrict__ content, uint64_t stride,
                                                  const uint64_t* __restrict__ sizes, uint64_t n,
                                                  uint64_t* __restrict__ keys, uint64_t* clk) {
  __shared__ uint32_t stack_lds[sdcas::SAMPLED_DEPTH][8][sdcas::SAMPLED_BLOCK];
  uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  const uint64_t f = (uint64_t)blockIdx.x * sdcas::SAMPLED_BLOCK + threadIdx.x;
  if (f < n) {
    const uint64_t g = (MODE == 0 || MODE == 4) ? f : (MODE == 1 ? (f & 31) : 0);
    sdcas::LdsStack<> stk{stack_lds, threadIdx.x};
    if (MODE == 5 || MODE == 6) {
      const uint4* q = reinterpret_cast<const uint4*>(content + (f >> 6) * 64 * stride) +
                       (MODE == 5 ? (f & 63) * 8 : (f & 63));
      keys[f] = MODE == 5 ? sdcas::cas_lane_sampled<false, sdcas::LAYOUT_LINE>(q, sizes[f], stk)
                          : sdcas::cas_lane_sampled<false, sdcas::LAYOUT_QUAD>(q, sizes[f], stk);
    } else {
      const uint4* q = reinterpret_cast<const uint4*>(content + g * stride);
      keys[f] = sdcas::cas_lane_sampled<MODE == 4>(q, sizes[f], stk);
    }
  }
  uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) {
    atomicAdd((unsigned long long*)&clk[0], (unsigned long long)(t1 - t0));
    atomicAdd((unsigned long long*)&clk[1], (unsigned long long)(r1 - r0));
  }
}

__global__ void __launch_bounds__(256) k_compress(uint32_t* out, uint32_t seed, uint64_t* clk) {
  uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  uint32_t cv[8];
  sdcas::set_iv(cv);
  uint32_t m[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) m[i] = threadIdx.x * 16 + i + seed;
  for (int i = 0; i < 953; ++i) {
    sdcas::compress(cv, m, (uint32_t)i, 0u, 64u, 0u);
    m[i & 15] ^= cv[0];
  }
  out[blockIdx.x * 256 + threadIdx.x] = cv[0] ^ cv[7];
  uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) {
    atomicAdd((unsigned long long*)&clk[0], (unsigned long long)(t1 - t0));
    atomicAdd((unsigned long long*)&clk[1], (unsigned long long)(r1 - r0));
  }
}

__global__ void fill_random(uint32_t* p, uint64_t nwords, uint32_t seed) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nwords;
       i += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t z = (i + seed) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    p[i] = (uint32_t)(z ^ (z >> 31));
  }
}

int main() {
  const uint64_t n = 1310720, stride = 57344;
  uint8_t* content;
  uint64_t *sizes, *keys, *clk;
  uint32_t* out;
  CHECK(hipMalloc(&content, n * stride));
  CHECK(hipMalloc(&sizes, n * 8));
  CHECK(hipMalloc(&keys, n * 8));
  CHECK(hipMalloc(&clk, 16));
  CHECK(hipMalloc(&out, n * 4));
  CHECK(hipMemset(content, 0x5a, n * stride));
  CHECK(hipMemset(sizes, 0x11, n * 8));
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  const char* names[] = {"K1 real (HBM)", "K1 window 32 files (L2)", "K1 broadcast", "compress-only x953",
                         "K1 real, nt loads", "K1 LINE-tiled layout", "K1 QUAD-tiled layout"};
  for (int data = 0; data < 2; ++data) {
  if (data == 1) {
    fill_random<<<4096, 256>>>((uint32_t*)content, n * stride / 4, 7u);
    CHECK(hipDeviceSynchronize());
  }
  printf("--- content: %s ---\n", data ? "random" : "constant 0x5a");
  for (int mode = 0; mode < 7; ++mode) {
    float best = 1e9;
    double ghz = 0;
    for (int rep = 0; rep < 4; ++rep) {
      CHECK(hipMemset(clk, 0, 16));
      (void)hipEventRecord(a, 0);
      const uint32_t blocks = (uint32_t)(n / 256);
      if (mode == 0) k1_variant<0><<<blocks, 256>>>(content, stride, sizes, n, keys, clk);
      if (mode == 1) k1_variant<1><<<blocks, 256>>>(content, stride, sizes, n, keys, clk);
      if (mode == 2) k1_variant<2><<<blocks, 256>>>(content, stride, sizes, n, keys, clk);
      if (mode == 3) k_compress<<<blocks, 256>>>(out, 1u, clk);
      if (mode == 4) k1_variant<4><<<blocks, 256>>>(content, stride, sizes, n, keys, clk);
      if (mode == 5) k1_variant<5><<<blocks, 256>>>(content, stride, sizes, n, keys, clk);
      if (mode == 6) k1_variant<6><<<blocks, 256>>>(content, stride, sizes, n, keys, clk);
      (void)hipEventRecord(b, 0);
      CHECK(hipEventSynchronize(b));
      float ms;
      (void)hipEventElapsedTime(&ms, a, b);
      uint64_t h[2];
      CHECK(hipMemcpy(h, clk, 16, hipMemcpyDeviceToHost));
      if (ms < best) { best = ms; ghz = (double)h[0] / (double)h[1] * 0.1; }
    }
    printf("%-28s %8.3f ms  %6.2f M files/s  clock %.3f GHz (s_memtime/s_memrealtime x 100 MHz)\n",
           names[mode], best, n / (best * 1e-3) / 1e6, ghz);
  }
  }
  return 0;
}
