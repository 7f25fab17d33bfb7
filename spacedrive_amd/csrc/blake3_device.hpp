// blake3_device.hpp — BLAKE3 compression for gfx950, written for the VALU.
//
// Replaces the compression inside the external `blake3` 1.5.0 crate that the reference
// calls from core/src/object/cas.rs:24-61 and core/src/object/validation/hash.rs:13-22.
// One 32-bit lane runs one compression: G is 2x v_add3_u32 + 2x v_add_u32 + 4x v_xor
// + 4x v_alignbit_b32 (rotate), so a full compression is ~680 VALU instructions with
// the message schedule resolved at compile time (no permutation moves).  There is no
// MFMA here: BLAKE3 is integer ARX, not a contraction.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace sdcas {

enum : uint32_t {
  CHUNK_START = 1u,
  CHUNK_END = 2u,
  PARENT = 4u,
  ROOT = 8u,
  BLOCK_LEN = 64u,
  CHUNK_LEN = 1024u,
};

__device__ constexpr uint32_t IV0 = 0x6A09E667u, IV1 = 0xBB67AE85u, IV2 = 0x3C6EF372u,
                              IV3 = 0xA54FF53Au, IV4 = 0x510E527Fu, IV5 = 0x9B05688Cu,
                              IV6 = 0x1F83D9ABu, IV7 = 0x5BE0CD19u;

// message word schedule per round (permutation applied r times), resolved at compile time
struct Sched {
  uint8_t s[7][16];
};
__host__ __device__ constexpr Sched make_sched() {
  Sched z{};
  const uint8_t perm[16] = {2, 6, 3, 10, 7, 0, 4, 13, 1, 11, 12, 5, 9, 14, 15, 8};
  for (int i = 0; i < 16; i++) z.s[0][i] = (uint8_t)i;
  for (int r = 1; r < 7; r++)
    for (int i = 0; i < 16; i++) z.s[r][i] = z.s[r - 1][perm[i]];
  return z;
}
constexpr Sched SCHED = make_sched();

__device__ __forceinline__ uint32_t rotr(uint32_t x, uint32_t n) {
  return __builtin_amdgcn_alignbit(x, x, n);
}

#define SDCAS_G(a, b, c, d, x, y)   \
  a = a + b + (x);                  \
  d = rotr(d ^ a, 16);              \
  c = c + d;                        \
  b = rotr(b ^ c, 12);              \
  a = a + b + (y);                  \
  d = rotr(d ^ a, 8);               \
  c = c + d;                        \
  b = rotr(b ^ c, 7);

template <int R>
__device__ __forceinline__ void round_fn(uint32_t& v0, uint32_t& v1, uint32_t& v2, uint32_t& v3,
                                         uint32_t& v4, uint32_t& v5, uint32_t& v6, uint32_t& v7,
                                         uint32_t& v8, uint32_t& v9, uint32_t& v10, uint32_t& v11,
                                         uint32_t& v12, uint32_t& v13, uint32_t& v14, uint32_t& v15,
                                         const uint32_t (&m)[16]) {
  constexpr const uint8_t* s = SCHED.s[R];
  SDCAS_G(v0, v4, v8, v12, m[s[0]], m[s[1]]);
  SDCAS_G(v1, v5, v9, v13, m[s[2]], m[s[3]]);
  SDCAS_G(v2, v6, v10, v14, m[s[4]], m[s[5]]);
  SDCAS_G(v3, v7, v11, v15, m[s[6]], m[s[7]]);
  SDCAS_G(v0, v5, v10, v15, m[s[8]], m[s[9]]);
  SDCAS_G(v1, v6, v11, v12, m[s[10]], m[s[11]]);
  SDCAS_G(v2, v7, v8, v13, m[s[12]], m[s[13]]);
  SDCAS_G(v3, v4, v9, v14, m[s[14]], m[s[15]]);
}

// cv <- first 8 output words of compress(cv, m, counter, blen, flags).
// counter_hi is always 0 on this path (chunk index < 2^32, i.e. files < 4 TiB per tree).
__device__ __forceinline__ void compress(uint32_t (&cv)[8], const uint32_t (&m)[16],
                                         uint32_t counter_lo, uint32_t counter_hi,
                                         uint32_t blen, uint32_t flags) {
  uint32_t v0 = cv[0], v1 = cv[1], v2 = cv[2], v3 = cv[3];
  uint32_t v4 = cv[4], v5 = cv[5], v6 = cv[6], v7 = cv[7];
  uint32_t v8 = IV0, v9 = IV1, v10 = IV2, v11 = IV3;
  uint32_t v12 = counter_lo, v13 = counter_hi, v14 = blen, v15 = flags;
  round_fn<0>(v0, v1, v2, v3, v4, v5, v6, v7, v8, v9, v10, v11, v12, v13, v14, v15, m);
  round_fn<1>(v0, v1, v2, v3, v4, v5, v6, v7, v8, v9, v10, v11, v12, v13, v14, v15, m);
  round_fn<2>(v0, v1, v2, v3, v4, v5, v6, v7, v8, v9, v10, v11, v12, v13, v14, v15, m);
  round_fn<3>(v0, v1, v2, v3, v4, v5, v6, v7, v8, v9, v10, v11, v12, v13, v14, v15, m);
  round_fn<4>(v0, v1, v2, v3, v4, v5, v6, v7, v8, v9, v10, v11, v12, v13, v14, v15, m);
  round_fn<5>(v0, v1, v2, v3, v4, v5, v6, v7, v8, v9, v10, v11, v12, v13, v14, v15, m);
  round_fn<6>(v0, v1, v2, v3, v4, v5, v6, v7, v8, v9, v10, v11, v12, v13, v14, v15, m);
  cv[0] = v0 ^ v8;  cv[1] = v1 ^ v9;  cv[2] = v2 ^ v10; cv[3] = v3 ^ v11;
  cv[4] = v4 ^ v12; cv[5] = v5 ^ v13; cv[6] = v6 ^ v14; cv[7] = v7 ^ v15;
}

__device__ __forceinline__ void set_iv(uint32_t (&cv)[8]) {
  cv[0] = IV0; cv[1] = IV1; cv[2] = IV2; cv[3] = IV3;
  cv[4] = IV4; cv[5] = IV5; cv[6] = IV6; cv[7] = IV7;
}

// parent node: cv <- compress(IV, left || right, 0, 64, PARENT | extra)
__device__ __forceinline__ void parent(uint32_t (&cv)[8], const uint32_t (&left)[8],
                                       const uint32_t (&right)[8], uint32_t extra_flags) {
  uint32_t m[16];
#pragma unroll
  for (int i = 0; i < 8; i++) { m[i] = left[i]; m[8 + i] = right[i]; }
  set_iv(cv);
  compress(cv, m, 0u, 0u, BLOCK_LEN, PARENT | extra_flags);
}

// cas key = big-endian u64 of the first 8 digest bytes (digest words are little-endian)
__device__ __forceinline__ uint64_t key_of(const uint32_t (&cv)[8]) {
  return ((uint64_t)__builtin_bswap32(cv[0]) << 32) | (uint64_t)__builtin_bswap32(cv[1]);
}

}  // namespace sdcas
