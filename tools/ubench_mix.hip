// ubench_mix.hip — gfx950 VALU issue: register-bank and rate-mixing effects that the
// single-op rates (ubench_valu.hip) do not show.  Every loop is one asm block over named
// VGPRs, so the register allocation (bank = vgpr index mod 4) is exactly what is written.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/ubench_mix tools/ubench_mix.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include "../spacedrive_amd/csrc/blake3_device.hpp"

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

constexpr int ITERS = 1024;  // x 32 instructions per iteration (.rept 4 of an 8-instr body)

#define CLOB "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48", "v49", "v50", \
  "v51", "v52", "v53", "v54", "v55", "v56", "v57", "v58", "v59", "v60", "v61", "v62", "v63", \
  "v64", "v65", "v66", "v67", "v68", "v69", "v70", "v71", "v72", "v73", "v74", "v75", "v76", \
  "v77", "v78", "v79", "s40", "scc"

// body: 8 instructions, independent destinations; INIT gives every register a value
#define KLOOP(NAME, BODY)                                                                     \
  __global__ void __launch_bounds__(256) NAME(uint32_t* out, uint32_t seed) {               \
    uint32_t r;                                                                               \
    asm volatile(                                                                             \
        ".irp i, 40,41,42,43,44,45,46,47,48,49,50,51,52,53,54,55,56,57,58,59,60,61,62,63,64,65,66,67,68,69,70,71,72,73,74,75,76,77,78,79\n" \
        "v_add_u32 v\\i, \\i, %1\n"                                                           \
        ".endr\n"                                                                             \
        "s_mov_b32 s40, %2\n"                                                                 \
        "1:\n"                                                                                \
        ".rept 4\n" BODY ".endr\n"                                                            \
        "s_sub_u32 s40, s40, 1\n"                                                             \
        "s_cmp_lg_u32 s40, 0\n"                                                               \
        "s_cbranch_scc1 1b\n"                                                                 \
        "v_xor_b32 %0, v40, v41\n"                                                            \
        "v_xor_b32 %0, %0, v42\n"                                                       \
        "v_xor_b32 %0, %0, v44\n"                                                       \
        "v_xor_b32 %0, %0, v48\n"                                                       \
        : "=v"(r) : "v"(threadIdx.x ^ seed), "s"(ITERS) : CLOB);                              \
    out[blockIdx.x * 256 + threadIdx.x] = r;                                                  \
  }

// add3: three distinct sources, all in bank 0 / in banks 0,1,2
KLOOP(k_add3_same, "v_add3_u32 v40, v40, v72, v76\n v_add3_u32 v44, v44, v72, v76\n v_add3_u32 v48, v48, v72, v76\n v_add3_u32 v52, v52, v72, v76\n"
                   "v_add3_u32 v56, v56, v72, v76\n v_add3_u32 v60, v60, v72, v76\n v_add3_u32 v64, v64, v72, v76\n v_add3_u32 v68, v68, v72, v76\n")
KLOOP(k_add3_diff, "v_add3_u32 v40, v40, v73, v78\n v_add3_u32 v44, v44, v73, v78\n v_add3_u32 v48, v48, v73, v78\n v_add3_u32 v52, v52, v73, v78\n"
                   "v_add3_u32 v56, v56, v73, v78\n v_add3_u32 v60, v60, v73, v78\n v_add3_u32 v64, v64, v73, v78\n v_add3_u32 v68, v68, v73, v78\n")
// two-source full-rate ops: same bank / different bank
KLOOP(k_xor_same, "v_xor_b32 v40, v40, v72\n v_xor_b32 v44, v44, v72\n v_xor_b32 v48, v48, v72\n v_xor_b32 v52, v52, v72\n"
                  "v_xor_b32 v56, v56, v72\n v_xor_b32 v60, v60, v72\n v_xor_b32 v64, v64, v72\n v_xor_b32 v68, v68, v72\n")
KLOOP(k_xor_diff, "v_xor_b32 v40, v40, v73\n v_xor_b32 v44, v44, v73\n v_xor_b32 v48, v48, v73\n v_xor_b32 v52, v52, v73\n"
                  "v_xor_b32 v56, v56, v73\n v_xor_b32 v60, v60, v73\n v_xor_b32 v64, v64, v73\n v_xor_b32 v68, v68, v73\n")
KLOOP(k_rot, "v_alignbit_b32 v40, v40, v40, 16\n v_alignbit_b32 v44, v44, v44, 16\n v_alignbit_b32 v48, v48, v48, 16\n v_alignbit_b32 v52, v52, v52, 16\n"
             "v_alignbit_b32 v56, v56, v56, 16\n v_alignbit_b32 v60, v60, v60, 16\n v_alignbit_b32 v64, v64, v64, 16\n v_alignbit_b32 v68, v68, v68, 16\n")
// rate mixing: 4 half-rate + 4 full-rate per body, interleaved / grouped
KLOOP(k_mix_inter, "v_alignbit_b32 v40, v40, v40, 16\n v_xor_b32 v44, v44, v73\n v_alignbit_b32 v48, v48, v48, 16\n v_xor_b32 v52, v52, v73\n"
                   "v_alignbit_b32 v56, v56, v56, 16\n v_xor_b32 v60, v60, v73\n v_alignbit_b32 v64, v64, v64, 16\n v_xor_b32 v68, v68, v73\n")
KLOOP(k_mix_group, "v_alignbit_b32 v40, v40, v40, 16\n v_alignbit_b32 v48, v48, v48, 16\n v_alignbit_b32 v56, v56, v56, 16\n v_alignbit_b32 v64, v64, v64, 16\n"
                   "v_xor_b32 v44, v44, v73\n v_xor_b32 v52, v52, v73\n v_xor_b32 v60, v60, v73\n v_xor_b32 v68, v68, v73\n")
// dependent pairs inside the body (G-like: xor feeding a rotate), 4 chains
KLOOP(k_xorrot_dep, "v_xor_b32 v40, v40, v73\n v_xor_b32 v44, v44, v73\n v_xor_b32 v48, v48, v73\n v_xor_b32 v52, v52, v73\n"
                    "v_alignbit_b32 v40, v40, v40, 16\n v_alignbit_b32 v44, v44, v44, 16\n v_alignbit_b32 v48, v48, v48, 16\n v_alignbit_b32 v52, v52, v52, 16\n")
// a full-rate VOP3 (e64) op mixed with alignbit
KLOOP(k_mix_e64, "v_alignbit_b32 v40, v40, v40, 16\n v_xor_b32_e64 v44, v44, v73\n v_alignbit_b32 v48, v48, v48, 16\n v_xor_b32_e64 v52, v52, v73\n"
                 "v_alignbit_b32 v56, v56, v56, 16\n v_xor_b32_e64 v60, v60, v73\n v_alignbit_b32 v64, v64, v64, 16\n v_xor_b32_e64 v68, v68, v73\n")
// add3 mixed with add
KLOOP(k_mix_add, "v_add3_u32 v40, v40, v73, v78\n v_add_u32 v44, v44, v73\n v_add3_u32 v48, v48, v73, v78\n v_add_u32 v52, v52, v73\n"
                 "v_add3_u32 v56, v56, v73, v78\n v_add_u32 v60, v60, v73\n v_add3_u32 v64, v64, v73, v78\n v_add_u32 v68, v68, v73\n")
// two full-rate adds in place of one add3 (a+b+m)
KLOOP(k_add2x, "v_add_u32 v40, v40, v73\n v_add_u32 v44, v44, v73\n v_add_u32 v48, v48, v73\n v_add_u32 v52, v52, v73\n"
               "v_add_u32 v40, v40, v78\n v_add_u32 v44, v44, v78\n v_add_u32 v48, v48, v78\n v_add_u32 v52, v52, v78\n")

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

// compute-only compression as K1 runs it (for the mixed-rate model check)
__global__ void __launch_bounds__(256) k_compress(uint32_t* out, uint32_t seed) {
  uint32_t cv[8];
  sdcas::set_iv(cv);
  uint32_t m[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) m[i] = threadIdx.x * 16 + i + seed;
  for (int i = 0; i < 64; ++i) {
    sdcas::compress(cv, m, (uint32_t)i, 0u, 64u, 0u);
    m[i & 15] ^= cv[0];
  }
  out[blockIdx.x * 256 + threadIdx.x] = cv[0] ^ cv[7];
}

// compress variants: the full-rate ops forced to VOP3 (e64) encodings or bitop3
__device__ __forceinline__ uint32_t xe(uint32_t a, uint32_t b) {
  uint32_t r; asm("v_xor_b32_e64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b)); return r; }
__device__ __forceinline__ uint32_t xb(uint32_t a, uint32_t b) {
  uint32_t r; asm("v_bitop3_b32 %0, %1, %2, 0 bitop3:0x96" : "=v"(r) : "v"(a), "v"(b)); return r; }
__device__ __forceinline__ uint32_t ae(uint32_t a, uint32_t b) {
  uint32_t r; asm("v_add_u32_e64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b)); return r; }
__device__ __forceinline__ uint32_t a2(uint32_t a, uint32_t b) { return a + b; }
__device__ __forceinline__ uint32_t x2(uint32_t a, uint32_t b) { return a ^ b; }
#define GV(XOR, ADD, a, b, c, d, x, y)                                           \
  a = a + b + (x); d = sdcas::rotr(XOR(d, a), 16); c = ADD(c, d);               \
  b = sdcas::rotr(XOR(b, c), 12); a = a + b + (y); d = sdcas::rotr(XOR(d, a), 8); \
  c = ADD(c, d); b = sdcas::rotr(XOR(b, c), 7);
#define COMPRESS_V(NAME, XOR, ADD)                                                         \
  __device__ __forceinline__ void NAME##_c(uint32_t (&cv)[8], const uint32_t (&m)[16], uint32_t ctr) { \
    uint32_t v0 = cv[0], v1 = cv[1], v2 = cv[2], v3 = cv[3], v4 = cv[4], v5 = cv[5], v6 = cv[6],  \
             v7 = cv[7], v8 = sdcas::IV0, v9 = sdcas::IV1, v10 = sdcas::IV2, v11 = sdcas::IV3,   \
             v12 = ctr, v13 = 0, v14 = 64, v15 = 0;                                              \
    _Pragma("unroll") for (int r = 0; r < 7; ++r) {                                              \
      const uint8_t* s = sdcas::SCHED.s[r];                                                       \
      GV(XOR, ADD, v0, v4, v8, v12, m[s[0]], m[s[1]]); GV(XOR, ADD, v1, v5, v9, v13, m[s[2]], m[s[3]]); \
      GV(XOR, ADD, v2, v6, v10, v14, m[s[4]], m[s[5]]); GV(XOR, ADD, v3, v7, v11, v15, m[s[6]], m[s[7]]); \
      GV(XOR, ADD, v0, v5, v10, v15, m[s[8]], m[s[9]]); GV(XOR, ADD, v1, v6, v11, v12, m[s[10]], m[s[11]]); \
      GV(XOR, ADD, v2, v7, v8, v13, m[s[12]], m[s[13]]); GV(XOR, ADD, v3, v4, v9, v14, m[s[14]], m[s[15]]); \
    }                                                                                              \
    cv[0] = XOR(v0, v8); cv[1] = XOR(v1, v9); cv[2] = XOR(v2, v10); cv[3] = XOR(v3, v11);          \
    cv[4] = XOR(v4, v12); cv[5] = XOR(v5, v13); cv[6] = XOR(v6, v14); cv[7] = XOR(v7, v15);        \
  }                                                                                                \
  __global__ void __launch_bounds__(256) NAME(uint32_t* out, uint32_t seed) {                     \
    uint32_t cv[8];                                                                                \
    sdcas::set_iv(cv);                                                                             \
    uint32_t m[16];                                                                                \
    _Pragma("unroll") for (int i = 0; i < 16; ++i) m[i] = threadIdx.x * 16 + i + seed;            \
    for (int i = 0; i < 64; ++i) { NAME##_c(cv, m, (uint32_t)i); m[i & 15] ^= cv[0]; }             \
    out[blockIdx.x * 256 + threadIdx.x] = cv[0] ^ cv[7];                                           \
  }
__device__ __forceinline__ uint32_t shr_(uint32_t a, uint32_t n) {
  uint32_t r; asm("v_lshrrev_b32 %0, %1, %2" : "=v"(r) : "i"(n), "v"(a)); return r; }
__device__ __forceinline__ uint32_t shl_(uint32_t a, uint32_t n) {
  uint32_t r; asm("v_lshlrev_b32 %0, %1, %2" : "=v"(r) : "i"(n), "v"(a)); return r; }
__device__ __forceinline__ uint32_t or_(uint32_t a, uint32_t b) {
  uint32_t r; asm("v_or_b32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b)); return r; }
__device__ __forceinline__ uint32_t add_(uint32_t a, uint32_t b) {
  uint32_t r; asm("v_add_u32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b)); return r; }
#define ROTSH(x, n) or_(shr_(x, n), shl_(x, 32 - n))
// G with every op full rate: a+b+m as two adds, rotations as shr/shl/or
#define GF(a, b, c, d, x, y)                                                              \
  a = add_(add_(a, x), b); d = ROTSH((d ^ a), 16); c = add_(c, d);                        \
  b = ROTSH((b ^ c), 12); a = add_(add_(a, y), b); d = ROTSH((d ^ a), 8);                \
  c = add_(c, d); b = ROTSH((b ^ c), 7);
// G with alignbit rotations but split adds
#define GS(a, b, c, d, x, y)                                                              \
  a = add_(add_(a, x), b); d = sdcas::rotr(d ^ a, 16); c = c + d;                         \
  b = sdcas::rotr(b ^ c, 12); a = add_(add_(a, y), b); d = sdcas::rotr(d ^ a, 8);        \
  c = c + d; b = sdcas::rotr(b ^ c, 7);
// G with shift rotations but add3
#define GR(a, b, c, d, x, y)                                                              \
  a = a + b + (x); d = ROTSH((d ^ a), 16); c = c + d;                                    \
  b = ROTSH((b ^ c), 12); a = a + b + (y); d = ROTSH((d ^ a), 8);                        \
  c = c + d; b = ROTSH((b ^ c), 7);
#define COMPRESS_G(NAME, G)                                                                 \
  __device__ __forceinline__ void NAME##_c(uint32_t (&cv)[8], const uint32_t (&m)[16], uint32_t ctr) { \
    uint32_t v0 = cv[0], v1 = cv[1], v2 = cv[2], v3 = cv[3], v4 = cv[4], v5 = cv[5], v6 = cv[6],  \
             v7 = cv[7], v8 = sdcas::IV0, v9 = sdcas::IV1, v10 = sdcas::IV2, v11 = sdcas::IV3,   \
             v12 = ctr, v13 = 0, v14 = 64, v15 = 0;                                              \
    _Pragma("unroll") for (int r = 0; r < 7; ++r) {                                              \
      const uint8_t* s = sdcas::SCHED.s[r];                                                       \
      G(v0, v4, v8, v12, m[s[0]], m[s[1]]); G(v1, v5, v9, v13, m[s[2]], m[s[3]]);                 \
      G(v2, v6, v10, v14, m[s[4]], m[s[5]]); G(v3, v7, v11, v15, m[s[6]], m[s[7]]);               \
      G(v0, v5, v10, v15, m[s[8]], m[s[9]]); G(v1, v6, v11, v12, m[s[10]], m[s[11]]);             \
      G(v2, v7, v8, v13, m[s[12]], m[s[13]]); G(v3, v4, v9, v14, m[s[14]], m[s[15]]);             \
    }                                                                                              \
    cv[0] = v0 ^ v8; cv[1] = v1 ^ v9; cv[2] = v2 ^ v10; cv[3] = v3 ^ v11;                          \
    cv[4] = v4 ^ v12; cv[5] = v5 ^ v13; cv[6] = v6 ^ v14; cv[7] = v7 ^ v15;                        \
  }                                                                                                \
  __global__ void __launch_bounds__(256) NAME(uint32_t* out, uint32_t seed) {                     \
    uint32_t cv[8];                                                                                \
    sdcas::set_iv(cv);                                                                             \
    uint32_t m[16];                                                                                \
    _Pragma("unroll") for (int i = 0; i < 16; ++i) m[i] = threadIdx.x * 16 + i + seed;            \
    for (int i = 0; i < 64; ++i) { NAME##_c(cv, m, (uint32_t)i); m[i & 15] ^= cv[0]; }             \
    out[blockIdx.x * 256 + threadIdx.x] = cv[0] ^ cv[7];                                           \
  }
COMPRESS_G(k_cg_full, GF)
COMPRESS_G(k_cg_split, GS)
COMPRESS_G(k_cg_shrot, GR)
COMPRESS_V(k_cv_plain, x2, a2)
COMPRESS_V(k_cv_xe, xe, a2)
COMPRESS_V(k_cv_xe_ae, xe, ae)
COMPRESS_V(k_cv_xb, xb, a2)
COMPRESS_V(k_cv_xb_ae, xb, ae)

int main() {
  hipDeviceProp_t p;
  CHECK(hipGetDeviceProperties(&p, 0));
  printf("device %s CUs %d\n", p.gcnArchName, p.multiProcessorCount);
  uint32_t* out;
  const double simds = p.multiProcessorCount * 4.0;
  CHECK(hipMalloc(&out, (size_t)p.multiProcessorCount * 64 * 256 * 4));
  struct { const char* n; void (*k)(uint32_t*, uint32_t); } ks[] = {
      {"add3 3 srcs same bank", k_add3_same}, {"add3 3 srcs banks 0,1,2", k_add3_diff},
      {"xor srcs same bank", k_xor_same}, {"xor srcs diff bank", k_xor_diff},
      {"alignbit x,x,16", k_rot}, {"alignbit/xor interleaved", k_mix_inter},
      {"4 alignbit then 4 xor", k_mix_group}, {"xor->rot dependent (4 chains)", k_xorrot_dep},
      {"alignbit/xor_e64 interleaved", k_mix_e64}, {"add3/add interleaved", k_mix_add},
      {"2x add (add3 split)", k_add2x}};
  for (int wps : {8}) {
    const int blocks = p.multiProcessorCount * wps;  // 256-thread block = 1 wave per SIMD
    printf("--- %d waves/SIMD ---\n", wps);
    for (auto& k : ks) {
      float ms = timeit(k.k, dim3(blocks), dim3(256), out);
      const double winstr = (double)blocks * 4 * ITERS * 32;
      const double rate = winstr / (ms * 1e-3) / simds / 1e9;
      printf("%-32s %8.3f ms  %.3f wave-instr/SIMD/ns\n", k.n, ms, rate);
    }
  }
  for (int wps : {4, 8}) {
    const int nb = p.multiProcessorCount * wps;
    float ms = timeit(k_compress, dim3(nb), dim3(256), out);
    const double comps = (double)nb * 256 * 64;
    printf("compress-only, %d waves/SIMD: %.3f ms  %.3e compressions/s -> %.1f M sampled files/s\n",
           wps, ms, comps / (ms * 1e-3), comps / (ms * 1e-3) / 953 / 1e6);
  }
  struct { const char* n; void (*k)(uint32_t*, uint32_t); } cs[] = {
      {"plain (compiler)", k_cv_plain}, {"xor e64", k_cv_xe}, {"xor e64 + add e64", k_cv_xe_ae},
      {"xor bitop3", k_cv_xb}, {"xor bitop3 + add e64", k_cv_xb_ae},
      {"ALL full-rate (2add, shr/shl/or)", k_cg_full}, {"alignbit + split adds", k_cg_split},
      {"shift rotations + add3", k_cg_shrot}};
  for (int wps : {2, 4, 8}) {
    const int nb = p.multiProcessorCount * wps;
    for (auto& k : cs) {
      float ms = timeit(k.k, dim3(nb), dim3(256), out);
      const double comps = (double)nb * 256 * 64;
      printf("compress %-34s %d w/SIMD: %.3f ms -> %.1f M sampled files/s\n", k.n, wps, ms,
             comps / (ms * 1e-3) / 953 / 1e6);
    }
  }
  return 0;
}
