// ubench_k1.hip — where K1 (sampled lane-per-file kernel) loses against the compute-only
// compression loop: the same lane code with its loads aimed at HBM (real layout), at an
// L2-resident window, or broadcast (every lane the same file), plus the compute-only loop,
// each with the shader clock measured inside the kernel (s_memtime / s_memrealtime).
// Build: hipcc --offload-arch=gfx950 -O3 -I spacedrive_amd/csrc -I include -o tools/ubench_k1 tools/ubench_k1.hip
// `ubench_k1 sustain <mode> <data> <seconds>` runs one variant back to back (tools/power_split.py).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../spacedrive_amd/csrc/cas_hash.hip"

// ---- the A/B-only variants of K1's lane program (moved out of the product, round 5) ------
// NT: non-temporal loads — measured 1.6x SLOWER (33.7 vs 55.0 M files/s): the 8 dwordx4
// loads of one 128-B line no longer share the line in L2 and each goes to HBM.
// Layouts of the sampled content in HBM (quad = 16 B; q points at the lane's first quad):
//   ROW   (0): file f at content + f*stride; quad i of pair P at q[8P + i]  (the product's)
//   LINE  (1): tiles of 64 files; pair P of lane l at tile + (64P + l)*128 B  -> q[512P + i]
//   QUAD  (2): tiles of 64 files; quad j of lane l at tile + (64j + l)*16 B    -> q[512P + 64i]
namespace ab {
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
enum : int { LAYOUT_ROW = 0, LAYOUT_LINE = 1, LAYOUT_QUAD = 2 };
template <int L> struct LayoutStride;
template <> struct LayoutStride<LAYOUT_ROW> { static constexpr uint32_t P = 8, I = 1; };
template <> struct LayoutStride<LAYOUT_LINE> { static constexpr uint32_t P = 512, I = 1; };
template <> struct LayoutStride<LAYOUT_QUAD> { static constexpr uint32_t P = 512, I = 64; };

template <bool NT, int L>
__device__ __forceinline__ void load_pair(const uint4* __restrict__ q, uint32_t P, uint4 (&buf)[8]) {
  const uint4* p = q + LayoutStride<L>::P * P;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    if (NT) {
      const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p + LayoutStride<L>::I * i));
      buf[i] = make_uint4(v.x, v.y, v.z, v.w);
    } else {
      buf[i] = p[LayoutStride<L>::I * i];
    }
  }
}

// the product's sdcas::cas_lane_sampled (cas_hash.hip, round 5's loop: both lines loaded at
// the iteration start) with the loader swapped — rebased in round 6: the round-5
// LINE / QUAD / non-temporal rows in profiles/r05/valu_power*/ubench_k1.txt were measured
// with the older loop that prefetched a pair across the back edge
template <bool NT = false, int L = LAYOUT_ROW, int BLK = 256>
__device__ __forceinline__ uint64_t cas_lane_sampled(const uint4* __restrict__ q, uint64_t size,
                                                     sdcas::LdsStack<BLK>& stk) {
  using namespace sdcas;
  uint32_t c0 = (uint32_t)size, c1 = (uint32_t)(size >> 32);
  uint4 A[8], B[8];
  uint32_t cv[8];
  for (uint32_t c = 0; c < SAMPLED_CHUNKS; ++c) {
    set_iv(cv);
#pragma unroll 1
    for (uint32_t pp = 0; pp < 4; ++pp) {
      const uint32_t P = 8u * c + 2u * pp;
      load_pair<NT, L>(q, P, A);
      load_pair<NT, L>(q, P + 1, B);
      compress_pair(cv, A, c0, c1, c, pp == 0 ? (uint32_t)CHUNK_START : 0u, 0u);
      compress_pair(cv, B, c0, c1, c, 0u, pp == 3 ? (uint32_t)CHUNK_END : 0u);
    }
    uint32_t total = c + 1;
    while ((total & 1u) == 0u) {
      uint32_t left[8];
      stk.pop(left);
      parent(cv, left, cv, 0u);
      total >>= 1;
    }
    stk.push(cv);
  }
  {
    const uint32_t m[16] = {c0, c1, 0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u};
    set_iv(cv);
    compress(cv, m, SAMPLED_CHUNKS, 0u, 8u, CHUNK_START | CHUNK_END);
  }
#pragma unroll
  for (int d = 0; d < 3; ++d) {
    uint32_t left[8];
    stk.pop(left);
    parent(cv, left, cv, d == 2 ? (uint32_t)ROOT : 0u);
  }
  return key_of(cv);
}
}  // namespace ab

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

// mode 0: real (file f), 1: window of 32 files (L2), 2: broadcast (file 0 for every lane),
// 4: real with non-temporal loads, 5: LINE-tiled layout (64-file tiles, 128-B lines
// interleaved), 6: QUAD-tiled layout (16-B quads interleaved: every load coalesced)
template <int MODE>
__global__ void __launch_bounds__(256) k1_variant(const uint8_t* __restrict__ content, uint64_t stride,
                                                  const uint64_t* __restrict__ sizes, uint64_t n,
                                                  uint64_t* __restrict__ keys, uint64_t* clk) {
  // 256-lane workgroups (the launch below): the stack is sized and the file indexed by the
  // workgroup's own width (indexing by the product's 512-lane SAMPLED_BLOCK skipped half the
  // files: the K1 rows of profiles/r05/valu_power/ubench_k1_halfgrid_bug.txt are 2x too fast;
  // its compute-only row, a separate kernel, is valid)
  __shared__ uint32_t stack_lds[sdcas::SAMPLED_DEPTH][8][256];
  uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  const uint64_t f = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (f < n) {
    const uint64_t g = (MODE == 0 || MODE == 4) ? f : (MODE == 1 ? (f & 31) : 0);
    sdcas::LdsStack<256> stk{stack_lds, threadIdx.x};
    if (MODE == 5 || MODE == 6) {
      const uint4* q = reinterpret_cast<const uint4*>(content + (f >> 6) * 64 * stride) +
                       (MODE == 5 ? (f & 63) * 8 : (f & 63));
      keys[f] = MODE == 5 ? ab::cas_lane_sampled<false, ab::LAYOUT_LINE>(q, sizes[f], stk)
                          : ab::cas_lane_sampled<false, ab::LAYOUT_QUAD>(q, sizes[f], stk);
    } else {
      const uint4* q = reinterpret_cast<const uint4*>(content + g * stride);
      keys[f] = ab::cas_lane_sampled<MODE == 4>(q, sizes[f], stk);
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

// compute-only with a CONSTANT message (the cv chain still evolves): the ALU share of the
// random-content power cost (tools/power_split.py)
__global__ void __launch_bounds__(256) k_compress_const(uint32_t* out, uint32_t seed, uint64_t* clk) {
  uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  uint32_t cv[8];
  sdcas::set_iv(cv);
  uint32_t m[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) m[i] = seed;
  for (int i = 0; i < 953; ++i) sdcas::compress(cv, m, (uint32_t)i, 0u, 64u, 0u);
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

static int launch(int mode, const uint8_t* content, uint64_t stride, const uint64_t* sizes, uint64_t n,
                  uint64_t* keys, uint32_t* out, uint64_t* clk) {
  const uint32_t blocks = (uint32_t)(n / 256);
  switch (mode) {
    case 0: k1_variant<0><<<blocks, 256>>>(content, stride, sizes, n, keys, clk); break;
    case 1: k1_variant<1><<<blocks, 256>>>(content, stride, sizes, n, keys, clk); break;
    case 2: k1_variant<2><<<blocks, 256>>>(content, stride, sizes, n, keys, clk); break;
    case 3: k_compress<<<blocks, 256>>>(out, 1u, clk); break;
    case 4: k1_variant<4><<<blocks, 256>>>(content, stride, sizes, n, keys, clk); break;
    case 5: k1_variant<5><<<blocks, 256>>>(content, stride, sizes, n, keys, clk); break;
    case 6: k1_variant<6><<<blocks, 256>>>(content, stride, sizes, n, keys, clk); break;
    case 7: k_compress_const<<<blocks, 256>>>(out, 0x5a5a5a5au, clk); break;
    default: return 1;
  }
  return 0;
}

// `ubench_k1 sustain <mode> <data> <seconds>`: one variant back to back for <seconds>
// (data 0: constant 0x5a bytes, 1: random, 2: zero), one JSON line with the rate and the
// in-kernel clock of the last second — tools/power_split.py samples rocm-smi beside it.
static int sustain(int mode, int data, double seconds) {
  const uint64_t n = 1310720, stride = 57344;
  uint8_t* content;
  uint64_t *sizes, *keys, *clk;
  uint32_t* out;
  CHECK(hipMalloc(&content, n * stride));
  CHECK(hipMalloc(&sizes, n * 8));
  CHECK(hipMalloc(&keys, n * 8));
  CHECK(hipMalloc(&clk, 16));
  CHECK(hipMalloc(&out, n * 4));
  CHECK(hipMemset(content, data == 2 ? 0 : 0x5a, n * stride));
  CHECK(hipMemset(sizes, 0x11, n * 8));
  if (data == 1) fill_random<<<4096, 256>>>((uint32_t*)content, n * stride / 4, 7u);
  CHECK(hipDeviceSynchronize());
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  double t_all = 0, t_late = 0, cyc = 0, real = 0;
  uint64_t launches = 0, late = 0;
  while (t_all < seconds * 1e3) {
    CHECK(hipMemset(clk, 0, 16));
    CHECK(hipEventRecord(a, 0));
    if (launch(mode, content, stride, sizes, n, keys, out, clk)) return 2;
    CHECK(hipEventRecord(b, 0));
    CHECK(hipEventSynchronize(b));
    float ms;
    CHECK(hipEventElapsedTime(&ms, a, b));
    t_all += ms;
    ++launches;
    if (t_all > 1e3) {  // after a 1 s settle
      uint64_t h[2];
      CHECK(hipMemcpy(h, clk, 16, hipMemcpyDeviceToHost));
      t_late += ms;
      ++late;
      cyc += (double)h[0];
      real += (double)h[1];
    }
  }
  printf("{\"mode\": %d, \"data\": %d, \"launches\": %llu, \"files_per_s\": %.1f, "
         "\"kernel_ms_mean\": %.4f, \"clock_ghz\": %.4f}\n",
         mode, data, (unsigned long long)launches, late ? n * late / (t_late * 1e-3) : 0.0,
         late ? t_late / late : 0.0, real > 0 ? cyc / real * 0.1 : 0.0);
  return 0;
}

int main(int argc, char** argv) {
  if (argc == 5 && !strcmp(argv[1], "sustain")) return sustain(atoi(argv[2]), atoi(argv[3]), atof(argv[4]));
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
