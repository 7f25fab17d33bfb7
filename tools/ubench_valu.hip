// ubench_valu.hip — gfx950 VALU microbenchmarks for the BLAKE3 ARX instruction mix.
// Measures, at full occupancy with 8 independent chains per lane, the throughput of each
// integer op K1 uses (and candidate replacements), plus the dependent-chain latency, and
// the compute-only rate of the real compression function (no memory traffic).
// Build: hipcc --offload-arch=gfx950 -O3 -o ubench tools/ubench_valu.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include "../spacedrive_amd/csrc/blake3_device.hpp"

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

constexpr int ITERS = 4096;

#define OP8(ASM)                                                                              \
  asm volatile(ASM : "+v"(a0) : "v"(b)); asm volatile(ASM : "+v"(a1) : "v"(b));             \
  asm volatile(ASM : "+v"(a2) : "v"(b)); asm volatile(ASM : "+v"(a3) : "v"(b));             \
  asm volatile(ASM : "+v"(a4) : "v"(b)); asm volatile(ASM : "+v"(a5) : "v"(b));             \
  asm volatile(ASM : "+v"(a6) : "v"(b)); asm volatile(ASM : "+v"(a7) : "v"(b));

#define KERNEL(NAME, ASM)                                                                     \
  __global__ void __launch_bounds__(256) NAME(uint32_t* out, uint32_t seed) {               \
    uint32_t a0 = threadIdx.x ^ seed, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4,    \
             a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7, b = seed * 3u + 1u;                        \
    for (int i = 0; i < ITERS; ++i) { OP8(ASM) }                                              \
    out[blockIdx.x * 256 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;              \
  }

KERNEL(k_xor, "v_xor_b32 %0, %0, %1")
KERNEL(k_add, "v_add_u32 %0, %0, %1")
KERNEL(k_add3, "v_add3_u32 %0, %0, %1, %0")
KERNEL(k_alignbit, "v_alignbit_b32 %0, %0, %0, 7")
KERNEL(k_xor3, "v_bitop3_b32 %0, %0, %1, %0 bitop3:0x96")
KERNEL(k_perm, "v_perm_b32 %0, %0, %0, %1")
KERNEL(k_lshlor, "v_lshl_or_b32 %0, %0, 7, %1")
KERNEL(k_xor_e64, "v_xor_b32_e64 %0, %0, %1")
KERNEL(k_pkadd16, "v_pk_add_u16 %0, %0, %1")
KERNEL(k_sdwa_hi, "v_xor_b32_sdwa %0, %0, %1 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_0")
KERNEL(k_sdwa_lo, "v_xor_b32_sdwa %0, %0, %1 dst_sel:WORD_0 dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:WORD_1")
KERNEL(k_sdwa_byte, "v_mov_b32_sdwa %0, %1 dst_sel:BYTE_3 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_0")
KERNEL(k_lshr, "v_lshrrev_b32 %0, 7, %0")
KERNEL(k_bfi, "v_bfi_b32 %0, %0, %1, %0")
KERNEL(k_or, "v_or_b32 %0, %0, %1")
KERNEL(k_add_e64, "v_add_u32_e64 %0, %0, %1")
KERNEL(k_lshladd, "v_lshl_add_u32 %0, %0, 7, %1")
KERNEL(k_alignbyte, "v_alignbyte_b32 %0, %0, %0, 2")
KERNEL(k_or3, "v_or3_b32 %0, %0, %1, %0")
KERNEL(k_andor, "v_and_or_b32 %0, %0, %1, %0")
KERNEL(k_mad24, "v_mad_u32_u24 %0, %0, %1, %0")
KERNEL(k_bitop3_16, "v_bitop3_b16 %0, %0, %1, %0 bitop3:0x96")

// operand-pattern variants of the half-rate ops (same reg twice vs distinct regs)
#define KERNEL3(NAME, ASM)                                                                    \
  __global__ void __launch_bounds__(256) NAME(uint32_t* out, uint32_t seed) {               \
    uint32_t a0 = threadIdx.x ^ seed, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4,    \
             a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7, b = seed * 3u + 1u, c = seed ^ 0x55u;     \
    for (int i = 0; i < ITERS; ++i) {                                                         \
      asm volatile(ASM : "+v"(a0) : "v"(b), "v"(c)); asm volatile(ASM : "+v"(a1) : "v"(b), "v"(c)); \
      asm volatile(ASM : "+v"(a2) : "v"(b), "v"(c)); asm volatile(ASM : "+v"(a3) : "v"(b), "v"(c)); \
      asm volatile(ASM : "+v"(a4) : "v"(b), "v"(c)); asm volatile(ASM : "+v"(a5) : "v"(b), "v"(c)); \
      asm volatile(ASM : "+v"(a6) : "v"(b), "v"(c)); asm volatile(ASM : "+v"(a7) : "v"(b), "v"(c)); \
    }                                                                                         \
    out[blockIdx.x * 256 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;              \
  }
KERNEL3(k_alignbit_2r, "v_alignbit_b32 %0, %0, %1, 7")
KERNEL3(k_alignbit_sh, "v_alignbit_b32 %0, %0, %0, %1")
KERNEL3(k_add3_3r, "v_add3_u32 %0, %0, %1, %2")
KERNEL3(k_bitop3_3r, "v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96")
KERNEL3(k_lshlor_3r, "v_lshl_or_b32 %0, %0, %1, %2")

// 64-bit register-pair ops (rotation as a 64-bit shift of a duplicated word)
#define KERNEL64(NAME, ASM)                                                                   \
  __global__ void __launch_bounds__(256) NAME(uint32_t* out, uint32_t seed) {               \
    uint64_t a[8];                                                                            \
    for (int j = 0; j < 8; ++j) a[j] = ((uint64_t)(threadIdx.x ^ seed) << 32) | (j + seed);  \
    uint64_t b = seed * 3u + 1u;                                                              \
    for (int i = 0; i < ITERS; ++i) {                                                         \
      asm volatile(ASM : "+v"(a[0]) : "v"(b)); asm volatile(ASM : "+v"(a[1]) : "v"(b));     \
      asm volatile(ASM : "+v"(a[2]) : "v"(b)); asm volatile(ASM : "+v"(a[3]) : "v"(b));     \
      asm volatile(ASM : "+v"(a[4]) : "v"(b)); asm volatile(ASM : "+v"(a[5]) : "v"(b));     \
      asm volatile(ASM : "+v"(a[6]) : "v"(b)); asm volatile(ASM : "+v"(a[7]) : "v"(b));     \
    }                                                                                         \
    uint64_t r = a[0] ^ a[1] ^ a[2] ^ a[3] ^ a[4] ^ a[5] ^ a[6] ^ a[7];                       \
    out[blockIdx.x * 256 + threadIdx.x] = (uint32_t)r ^ (uint32_t)(r >> 32);                  \
  }
KERNEL64(k_lshr64, "v_lshrrev_b64 %0, 7, %0")
KERNEL64(k_pkmov, "v_pk_mov_b32 %0, %0, %1 op_sel:[1,0]")
KERNEL64(k_lshladd64, "v_lshl_add_u64 %0, %0, 0, %1")

// dependent chain: one accumulator
__global__ void __launch_bounds__(64) k_dep_alignbit(uint32_t* out, uint32_t seed) {
  uint32_t a = threadIdx.x ^ seed;
  for (int i = 0; i < ITERS * 8; ++i) asm volatile("v_alignbit_b32 %0, %0, %0, 7" : "+v"(a));
  out[blockIdx.x * 64 + threadIdx.x] = a;
}
__global__ void __launch_bounds__(64) k_dep_xor(uint32_t* out, uint32_t seed) {
  uint32_t a = threadIdx.x ^ seed, b = seed;
  for (int i = 0; i < ITERS * 8; ++i) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a) : "v"(b));
  out[blockIdx.x * 64 + threadIdx.x] = a;
}

// compute-only compression: the real compress() on register data, 64 compressions/lane
__global__ void __launch_bounds__(256) k_compress(uint32_t* out, uint32_t seed) {
  uint32_t cv[8];
  sdcas::set_iv(cv);
  uint32_t m[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) m[i] = threadIdx.x * 16 + i + seed;
  for (int i = 0; i < 64; ++i) {
    sdcas::compress(cv, m, (uint32_t)i, 0u, 64u, 0u);
    m[i & 15] ^= cv[0];  // keep the chain live without changing the instruction mix much
  }
  out[blockIdx.x * 256 + threadIdx.x] = cv[0] ^ cv[7];
}

// variant: a + b + x as two full-rate adds, the message add first (off the a->b chain)
__device__ __forceinline__ uint32_t add2(uint32_t a, uint32_t b) {
  uint32_t r;
  asm volatile("v_add_u32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
#define G2(a, b, c, d, x, y)                                        \
  a = add2(add2(a, x), b); d = sdcas::rotr(d ^ a, 16); c = c + d;   \
  b = sdcas::rotr(b ^ c, 12); a = add2(add2(a, y), b);              \
  d = sdcas::rotr(d ^ a, 8); c = c + d; b = sdcas::rotr(b ^ c, 7);
__device__ __forceinline__ void compress2(uint32_t (&cv)[8], const uint32_t (&m)[16], uint32_t ctr) {
  uint32_t v0 = cv[0], v1 = cv[1], v2 = cv[2], v3 = cv[3], v4 = cv[4], v5 = cv[5], v6 = cv[6],
           v7 = cv[7], v8 = sdcas::IV0, v9 = sdcas::IV1, v10 = sdcas::IV2, v11 = sdcas::IV3,
           v12 = ctr, v13 = 0, v14 = 64, v15 = 0;
#pragma unroll
  for (int r = 0; r < 7; ++r) {
    const uint8_t* s = sdcas::SCHED.s[r];
    G2(v0, v4, v8, v12, m[s[0]], m[s[1]]); G2(v1, v5, v9, v13, m[s[2]], m[s[3]]);
    G2(v2, v6, v10, v14, m[s[4]], m[s[5]]); G2(v3, v7, v11, v15, m[s[6]], m[s[7]]);
    G2(v0, v5, v10, v15, m[s[8]], m[s[9]]); G2(v1, v6, v11, v12, m[s[10]], m[s[11]]);
    G2(v2, v7, v8, v13, m[s[12]], m[s[13]]); G2(v3, v4, v9, v14, m[s[14]], m[s[15]]);
  }
  cv[0] = v0 ^ v8; cv[1] = v1 ^ v9; cv[2] = v2 ^ v10; cv[3] = v3 ^ v11;
  cv[4] = v4 ^ v12; cv[5] = v5 ^ v13; cv[6] = v6 ^ v14; cv[7] = v7 ^ v15;
}
__global__ void __launch_bounds__(256) k_compress2(uint32_t* out, uint32_t seed) {
  uint32_t cv[8];
  sdcas::set_iv(cv);
  uint32_t m[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) m[i] = threadIdx.x * 16 + i + seed;
  for (int i = 0; i < 64; ++i) {
    compress2(cv, m, (uint32_t)i);
    m[i & 15] ^= cv[0];
  }
  out[blockIdx.x * 256 + threadIdx.x] = cv[0] ^ cv[7];
}

template <typename K>
static float timeit(K kern, dim3 grid, dim3 block, uint32_t* out) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  hipLaunchKernelGGL(kern, grid, block, 0, 0, out, 1u);  // warm
  (void)hipDeviceSynchronize();
  (void)hipEventRecord(a, 0);
  for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(kern, grid, block, 0, 0, out, (uint32_t)r);
  (void)hipEventRecord(b, 0);
  (void)hipEventSynchronize(b);
  float ms;
  (void)hipEventElapsedTime(&ms, a, b);
  return ms / 5;
}

int main() {
  hipDeviceProp_t p;
  CHECK(hipGetDeviceProperties(&p, 0));
  printf("device %s CUs %d clock %d kHz\n", p.gcnArchName, p.multiProcessorCount, p.clockRate);
  uint32_t* out;
  const int blocks = p.multiProcessorCount * 8 * 4;  // 32 waves/CU worth of 256-thread blocks
  CHECK(hipMalloc(&out, (size_t)blocks * 256 * 4));
  const double simds = p.multiProcessorCount * 4.0;
  struct { const char* n; void (*k)(uint32_t*, uint32_t); } ks[] = {
      {"v_xor_b32 (VOP2)", k_xor}, {"v_add_u32 (VOP2)", k_add}, {"v_add3_u32", k_add3},
      {"v_alignbit_b32", k_alignbit}, {"v_bitop3_b32 (xor3)", k_xor3}, {"v_perm_b32", k_perm},
      {"v_lshl_or_b32", k_lshlor}, {"v_xor_b32_e64 (VOP3 enc)", k_xor_e64},
      {"v_pk_add_u16", k_pkadd16},
      {"v_xor_b32_sdwa WORD_1<-WORD_0", k_sdwa_hi}, {"v_xor_b32_sdwa WORD_0<-WORD_1", k_sdwa_lo},
      {"v_mov_b32_sdwa BYTE_3<-BYTE_0", k_sdwa_byte}, {"v_lshrrev_b32", k_lshr},
      {"v_bfi_b32", k_bfi}, {"v_or_b32", k_or},
      {"v_add_u32_e64", k_add_e64}, {"v_lshl_add_u32", k_lshladd},
      {"v_alignbyte_b32", k_alignbyte}, {"v_or3_b32", k_or3}, {"v_and_or_b32", k_andor},
      {"v_mad_u32_u24", k_mad24}, {"v_bitop3_b16", k_bitop3_16},
      {"v_alignbit_b32 a,a,b,7", k_alignbit_2r}, {"v_alignbit_b32 a,a,a,vS", k_alignbit_sh},
      {"v_add3_u32 a,a,b,c", k_add3_3r}, {"v_bitop3_b32 a,a,b,c", k_bitop3_3r},
      {"v_lshl_or_b32 a,a,b,c", k_lshlor_3r},
      {"v_lshrrev_b64", k_lshr64}, {"v_pk_mov_b32", k_pkmov}, {"v_lshl_add_u64", k_lshladd64}};
  for (auto& k : ks) {
    float ms = timeit(k.k, dim3(blocks), dim3(256), out);
    const double winstr = (double)blocks * 4 * ITERS * 8;  // wave-instructions
    const double rate = winstr / (ms * 1e-3);
    printf("%-28s %8.3f ms  %.3e wave-instr/s  = %.3f wave-instr/SIMD/ns  (2.4GHz full rate = 1.2)\n",
           k.n, ms, rate, rate / simds / 1e9);
  }
  {
    float ms = timeit(k_dep_alignbit, dim3(p.multiProcessorCount * 4), dim3(64), out);
    printf("dep chain alignbit, 1 wave/SIMD: %.2f ns/instr\n", ms * 1e6 / (ITERS * 8));
    ms = timeit(k_dep_xor, dim3(p.multiProcessorCount * 4), dim3(64), out);
    printf("dep chain xor, 1 wave/SIMD: %.2f ns/instr\n", ms * 1e6 / (ITERS * 8));
  }
  for (int wps : {1, 2, 3, 4, 8}) {  // waves per SIMD
    const int nb = p.multiProcessorCount * wps;  // 256-thread blocks = 4 waves = 1 per SIMD
    float ms = timeit(k_compress, dim3(nb), dim3(256), out);
    const double comps = (double)nb * 256 * 64;
    printf("compress-only, %d waves/SIMD: %.3f ms  %.3e compressions/s  -> %.1f M sampled files/s (953 each)\n",
           wps, ms, comps / (ms * 1e-3), comps / (ms * 1e-3) / 953 / 1e6);
  }
  for (int wps : {1, 4, 8}) {
    const int nb = p.multiProcessorCount * wps;
    float ms = timeit(k_compress2, dim3(nb), dim3(256), out);
    const double comps = (double)nb * 256 * 64;
    printf("compress-only (add3 split), %d waves/SIMD: %.3f ms  -> %.1f M sampled files/s\n",
           wps, ms, comps / (ms * 1e-3) / 953 / 1e6);
  }
  return 0;
}
