/*
 * cas_fast.c — SIMD CPU baseline for cas_id hashing.  TEST/BASELINE INFRASTRUCTURE ONLY
 * (bench.py's cpu_baseline leg; see oracle.h).
 *
 * The reference hashes each file with the `blake3` 1.5.0 crate, whose AVX-512 path
 * (`hash_many`) compresses 16 independent chunks per zmm lane group.  This baseline
 * gives the CPU the same SIMD width: 16 files per lane group, one file per 32-bit
 * lane, BLAKE3 chaining-value stack per lane (same tree as blake3_ref.c), so the GPU
 * is compared against a SIMD host, not a scalar strawman.  A group of files of unequal
 * length is hashed file by file, chunk-parallel (16 chunks of one file per lane group,
 * as the crate's `hash_many` does for one input).  Hosts without AVX-512F use the
 * scalar path everywhere.  Results are checked against blake3_ref.c by tests.
 */
#define _GNU_SOURCE
#include <immintrin.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

#define AVX512 __attribute__((target("avx512f")))

static const uint32_t IV32[8] = {0x6A09E667u, 0xBB67AE85u, 0x3C6EF372u, 0xA54FF53Au,
                                 0x510E527Fu, 0x9B05688Cu, 0x1F83D9ABu, 0x5BE0CD19u};

#define ROT(x, n) _mm512_ror_epi32((x), (n))
#define G(a, b, c, d, x, y)                       \
  do {                                            \
    a = _mm512_add_epi32(_mm512_add_epi32(a, b), x); \
    d = ROT(_mm512_xor_si512(d, a), 16);          \
    c = _mm512_add_epi32(c, d);                   \
    b = ROT(_mm512_xor_si512(b, c), 12);          \
    a = _mm512_add_epi32(_mm512_add_epi32(a, b), y); \
    d = ROT(_mm512_xor_si512(d, a), 8);           \
    c = _mm512_add_epi32(c, d);                   \
    b = ROT(_mm512_xor_si512(b, c), 7);           \
  } while (0)

static const uint8_t SCHED[7][16] = {
    {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15},
    {2, 6, 3, 10, 7, 0, 4, 13, 1, 11, 12, 5, 9, 14, 15, 8},
    {3, 4, 10, 12, 13, 2, 7, 14, 6, 5, 9, 0, 11, 15, 8, 1},
    {10, 7, 12, 9, 14, 3, 13, 15, 4, 0, 11, 2, 5, 8, 1, 6},
    {12, 13, 9, 11, 15, 10, 14, 8, 7, 2, 5, 3, 0, 1, 6, 4},
    {9, 14, 11, 5, 8, 12, 15, 1, 13, 3, 0, 10, 2, 6, 4, 7},
    {11, 15, 5, 0, 1, 9, 8, 6, 14, 10, 2, 12, 3, 4, 7, 13},
};

/* cv[8] <- first 8 words of compress(cv, m, counter (per-lane lo, hi = 0), blen, flags) */
AVX512 static inline void compress16(__m512i cv[8], const __m512i m[16], __m512i ctr_lo,
                                     uint32_t blen, uint32_t flags, __m512i out_hi[8]) {
  __m512i s0 = cv[0], s1 = cv[1], s2 = cv[2], s3 = cv[3], s4 = cv[4], s5 = cv[5], s6 = cv[6], s7 = cv[7];
  __m512i s8 = _mm512_set1_epi32((int)IV32[0]), s9 = _mm512_set1_epi32((int)IV32[1]);
  __m512i s10 = _mm512_set1_epi32((int)IV32[2]), s11 = _mm512_set1_epi32((int)IV32[3]);
  __m512i s12 = ctr_lo, s13 = _mm512_setzero_si512();
  __m512i s14 = _mm512_set1_epi32((int)blen), s15 = _mm512_set1_epi32((int)flags);
  for (int r = 0; r < 7; r++) {
    const uint8_t* z = SCHED[r];
    G(s0, s4, s8, s12, m[z[0]], m[z[1]]);
    G(s1, s5, s9, s13, m[z[2]], m[z[3]]);
    G(s2, s6, s10, s14, m[z[4]], m[z[5]]);
    G(s3, s7, s11, s15, m[z[6]], m[z[7]]);
    G(s0, s5, s10, s15, m[z[8]], m[z[9]]);
    G(s1, s6, s11, s12, m[z[10]], m[z[11]]);
    G(s2, s7, s8, s13, m[z[12]], m[z[13]]);
    G(s3, s4, s9, s14, m[z[14]], m[z[15]]);
  }
  cv[0] = _mm512_xor_si512(s0, s8); cv[1] = _mm512_xor_si512(s1, s9);
  cv[2] = _mm512_xor_si512(s2, s10); cv[3] = _mm512_xor_si512(s3, s11);
  cv[4] = _mm512_xor_si512(s4, s12); cv[5] = _mm512_xor_si512(s5, s13);
  cv[6] = _mm512_xor_si512(s6, s14); cv[7] = _mm512_xor_si512(s7, s15);
  (void)out_hi;
}

/* 16x16 u32 transpose: rows r[i] (lane i's 16 words) -> m[w] (word w of every lane) */
AVX512 static inline void transpose16(__m512i r[16]) {
  __m512i t[16];
  for (int i = 0; i < 16; i += 2) {
    t[i] = _mm512_unpacklo_epi32(r[i], r[i + 1]);
    t[i + 1] = _mm512_unpackhi_epi32(r[i], r[i + 1]);
  }
  for (int i = 0; i < 16; i += 4) {
    r[i] = _mm512_unpacklo_epi64(t[i], t[i + 2]);
    r[i + 1] = _mm512_unpackhi_epi64(t[i], t[i + 2]);
    r[i + 2] = _mm512_unpacklo_epi64(t[i + 1], t[i + 3]);
    r[i + 3] = _mm512_unpackhi_epi64(t[i + 1], t[i + 3]);
  }
  /* now r[4g + k] holds, per 128-bit lane q, words (4q..4q+3 of row group g) for word k */
  for (int k = 0; k < 4; k++) {
    t[k] = _mm512_shuffle_i32x4(r[k], r[4 + k], 0x88);
    t[4 + k] = _mm512_shuffle_i32x4(r[k], r[4 + k], 0xdd);
    t[8 + k] = _mm512_shuffle_i32x4(r[8 + k], r[12 + k], 0x88);
    t[12 + k] = _mm512_shuffle_i32x4(r[8 + k], r[12 + k], 0xdd);
  }
  for (int k = 0; k < 4; k++) {
    r[k] = _mm512_shuffle_i32x4(t[k], t[8 + k], 0x88);
    r[8 + k] = _mm512_shuffle_i32x4(t[k], t[8 + k], 0xdd);
    r[4 + k] = _mm512_shuffle_i32x4(t[4 + k], t[12 + k], 0x88);
    r[12 + k] = _mm512_shuffle_i32x4(t[4 + k], t[12 + k], 0xdd);
  }
}

/* Hash 16 cas messages le64(size[l]) || content[l][0..clen), equal clen. */
AVX512 static void cas16(const uint8_t* const content[16], const uint64_t size[16], size_t clen,
                         uint64_t out[16]) {
  const uint64_t mlen = clen + 8;
  const uint64_t nchunks = mlen <= 1024 ? 1 : (mlen + 1023) / 1024;
  __m512i stack[8][8];
  int sp = 0;
  const __m512i iv[8] = {
      _mm512_set1_epi32((int)IV32[0]), _mm512_set1_epi32((int)IV32[1]), _mm512_set1_epi32((int)IV32[2]),
      _mm512_set1_epi32((int)IV32[3]), _mm512_set1_epi32((int)IV32[4]), _mm512_set1_epi32((int)IV32[5]),
      _mm512_set1_epi32((int)IV32[6]), _mm512_set1_epi32((int)IV32[7])};
  __m512i cv[8] = {iv[0], iv[1], iv[2], iv[3], iv[4], iv[5], iv[6], iv[7]};
  uint8_t tmp[16][64] __attribute__((aligned(64)));
  for (uint64_t c = 0; c < nchunks; c++) {
    const int last = (c + 1 == nchunks);
    const uint64_t cbytes = last ? mlen - c * 1024 : 1024;
    const uint64_t nblk = cbytes == 0 ? 1 : (cbytes + 63) / 64;
    for (int i = 0; i < 8; i++) cv[i] = iv[i];
    const __m512i ctr = _mm512_set1_epi32((int)(uint32_t)c);
    for (uint64_t b = 0; b < nblk; b++) {
      const uint64_t moff = c * 1024 + b * 64; /* message offset of this block */
      const uint64_t blen = (mlen - moff) < 64 ? (mlen - moff) : 64;
      __m512i r[16];
      if (moff >= 8 && moff + 64 <= mlen) {
        for (int l = 0; l < 16; l++) r[l] = _mm512_loadu_si512((const void*)(content[l] + moff - 8));
      } else {
        for (int l = 0; l < 16; l++) {
          memset(tmp[l], 0, 64);
          for (uint64_t k = 0; k < blen; k++) {
            uint64_t p = moff + k;
            tmp[l][k] = p < 8 ? (uint8_t)(size[l] >> (8 * p)) : content[l][p - 8];
          }
          r[l] = _mm512_load_si512((const void*)tmp[l]);
        }
      }
      transpose16(r);
      uint32_t flags = (b == 0 ? 1u : 0u) | (b + 1 == nblk ? 2u : 0u);
      if (last && nchunks == 1 && b + 1 == nblk) flags |= 8u;
      compress16(cv, r, ctr, (uint32_t)blen, flags, NULL);
    }
    if (!last) {
      uint64_t total = c + 1;
      while ((total & 1) == 0) {
        __m512i m[16];
        --sp;
        for (int i = 0; i < 8; i++) { m[i] = stack[sp][i]; m[8 + i] = cv[i]; cv[i] = iv[i]; }
        compress16(cv, m, _mm512_setzero_si512(), 64, 4u, NULL);
        total >>= 1;
      }
      for (int i = 0; i < 8; i++) stack[sp][i] = cv[i];
      sp++;
    }
  }
  while (sp > 0) {
    __m512i m[16];
    --sp;
    for (int i = 0; i < 8; i++) { m[i] = stack[sp][i]; m[8 + i] = cv[i]; cv[i] = iv[i]; }
    compress16(cv, m, _mm512_setzero_si512(), 64, 4u | (sp == 0 ? 8u : 0u), NULL);
  }
  uint32_t w0[16], w1[16];
  _mm512_storeu_si512((void*)w0, cv[0]);
  _mm512_storeu_si512((void*)w1, cv[1]);
  for (int l = 0; l < 16; l++)
    out[l] = ((uint64_t)__builtin_bswap32(w0[l]) << 32) | __builtin_bswap32(w1[l]);
}

/* compress16 with per-lane block length and flags; lanes outside `active` keep cv. */
AVX512 static inline void compress16v(__m512i cv[8], const __m512i m[16], __m512i ctr_lo,
                                      __m512i blen, __m512i flags, __mmask16 active) {
  __m512i s0 = cv[0], s1 = cv[1], s2 = cv[2], s3 = cv[3], s4 = cv[4], s5 = cv[5], s6 = cv[6], s7 = cv[7];
  __m512i s8 = _mm512_set1_epi32((int)IV32[0]), s9 = _mm512_set1_epi32((int)IV32[1]);
  __m512i s10 = _mm512_set1_epi32((int)IV32[2]), s11 = _mm512_set1_epi32((int)IV32[3]);
  __m512i s12 = ctr_lo, s13 = _mm512_setzero_si512(), s14 = blen, s15 = flags;
  for (int r = 0; r < 7; r++) {
    const uint8_t* z = SCHED[r];
    G(s0, s4, s8, s12, m[z[0]], m[z[1]]);
    G(s1, s5, s9, s13, m[z[2]], m[z[3]]);
    G(s2, s6, s10, s14, m[z[4]], m[z[5]]);
    G(s3, s7, s11, s15, m[z[6]], m[z[7]]);
    G(s0, s5, s10, s15, m[z[8]], m[z[9]]);
    G(s1, s6, s11, s12, m[z[10]], m[z[11]]);
    G(s2, s7, s8, s13, m[z[12]], m[z[13]]);
    G(s3, s4, s9, s14, m[z[14]], m[z[15]]);
  }
  cv[0] = _mm512_mask_xor_epi32(cv[0], active, s0, s8); cv[1] = _mm512_mask_xor_epi32(cv[1], active, s1, s9);
  cv[2] = _mm512_mask_xor_epi32(cv[2], active, s2, s10); cv[3] = _mm512_mask_xor_epi32(cv[3], active, s3, s11);
  cv[4] = _mm512_mask_xor_epi32(cv[4], active, s4, s12); cv[5] = _mm512_mask_xor_epi32(cv[5], active, s5, s13);
  cv[6] = _mm512_mask_xor_epi32(cv[6], active, s6, s14); cv[7] = _mm512_mask_xor_epi32(cv[7], active, s7, s15);
}

/* One cas message hashed chunk-parallel, the way the blake3 crate's `hash_many` hashes one
 * input: 16 chunks per lane group (the partial last chunk rides in the last group as a
 * masked lane), then the parent levels 16 pairs at a time (level-wise pair-and-promote ==
 * the left-balanced tree).  Messages of one chunk and of more than 128 chunks use the
 * scalar restatement. */
#define CP_MAX 128
AVX512 static uint64_t cas_chunkpar16(const uint8_t* content, size_t clen, uint64_t size) {
  const uint64_t mlen = (uint64_t)clen + 8;
  const uint64_t nchunks = (mlen + 1023) / 1024;
  if (nchunks <= 1 || nchunks > CP_MAX) return orc_cas_key(content, clen, size);
  uint8_t head[1024] __attribute__((aligned(64)));
  uint8_t tail[1024] __attribute__((aligned(64)));
  memcpy(head, &size, 8); /* le64(size): x86 is little-endian */
  memcpy(head + 8, content, 1016);
  const uint64_t tlen = mlen - (nchunks - 1) * 1024; /* 1..1024 bytes in the last chunk */
  memset(tail, 0, sizeof tail);
  memcpy(tail, content + (nchunks - 1) * 1024 - 8, tlen);
  const uint32_t tblk = (uint32_t)((tlen + 63) / 64);
  uint32_t cvs[2][CP_MAX][8] __attribute__((aligned(64)));
  const __m512i lane = _mm512_setr_epi32(0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15);
  for (uint64_t c0 = 0; c0 < nchunks; c0 += 16) {
    const uint8_t* ptr[16];
    uint32_t nblk[16];
    for (int l = 0; l < 16; l++) {
      const uint64_t c = c0 + (uint64_t)l < nchunks ? c0 + (uint64_t)l : c0;
      ptr[l] = c == 0 ? head : (c + 1 == nchunks ? tail : content + c * 1024 - 8);
      nblk[l] = c0 + (uint64_t)l >= nchunks ? 0 : (c + 1 == nchunks ? tblk : 16);
    }
    const __m512i vnblk = _mm512_loadu_si512((const void*)nblk);
    const __m512i ctr = _mm512_add_epi32(_mm512_set1_epi32((int)c0), lane);
    __m512i cv[8];
    for (int i = 0; i < 8; i++) cv[i] = _mm512_set1_epi32((int)IV32[i]);
    for (uint32_t b = 0; b < 16; b++) {
      const __m512i vb = _mm512_set1_epi32((int)b);
      const __mmask16 act = _mm512_cmplt_epu32_mask(vb, vnblk);
      if (!act) break;
      const __mmask16 end = _mm512_cmpeq_epi32_mask(_mm512_add_epi32(vb, _mm512_set1_epi32(1)), vnblk);
      const __m512i last_len = _mm512_mask_blend_epi32((__mmask16)(1u << (nchunks - 1 - c0 < 16 ? nchunks - 1 - c0 : 16)),
                                                       _mm512_set1_epi32(64),
                                                       _mm512_set1_epi32((int)(tlen - 64 * (tblk - 1))));
      const __m512i blen = _mm512_mask_blend_epi32(end, _mm512_set1_epi32(64), last_len);
      __m512i flags = _mm512_mask_blend_epi32(end, _mm512_setzero_si512(), _mm512_set1_epi32(2));
      if (b == 0) flags = _mm512_or_si512(flags, _mm512_set1_epi32(1));
      __m512i r[16];
      for (int l = 0; l < 16; l++)
        r[l] = _mm512_loadu_si512((const void*)(ptr[l] + 64 * (b < nblk[l] ? b : 0)));
      transpose16(r);
      compress16v(cv, r, ctr, blen, flags, act);
    }
    uint32_t w[8][16] __attribute__((aligned(64)));
    for (int i = 0; i < 8; i++) _mm512_store_si512((void*)w[i], cv[i]);
    for (int l = 0; l < 16 && c0 + (uint64_t)l < nchunks; l++)
      for (int i = 0; i < 8; i++) cvs[0][c0 + (uint64_t)l][i] = w[i][l];
  }
  /* parent levels, 16 pairs per compression group */
  uint32_t count = (uint32_t)nchunks;
  int cur = 0;
  while (count > 1) {
    const uint32_t pairs = count / 2;
    const uint32_t flags = 4u | (count == 2 ? 8u : 0u);
    for (uint32_t p0 = 0; p0 < pairs; p0 += 16) {
      const __m512i pidx = _mm512_min_epu32(_mm512_add_epi32(_mm512_set1_epi32((int)p0), lane),
                                            _mm512_set1_epi32((int)(pairs - 1)));
      const __m512i base = _mm512_mullo_epi32(pidx, _mm512_set1_epi32(16)); /* 2 cvs x 8 words */
      __m512i m[16], cv[8];
      for (int i = 0; i < 16; i++)
        m[i] = _mm512_i32gather_epi32(_mm512_add_epi32(base, _mm512_set1_epi32(i)),
                                      (const void*)cvs[cur], 4);
      for (int i = 0; i < 8; i++) cv[i] = _mm512_set1_epi32((int)IV32[i]);
      compress16v(cv, m, _mm512_setzero_si512(), _mm512_set1_epi32(64), _mm512_set1_epi32((int)flags),
                  (__mmask16)0xFFFF);
      uint32_t w[8][16] __attribute__((aligned(64)));
      for (int i = 0; i < 8; i++) _mm512_store_si512((void*)w[i], cv[i]);
      for (uint32_t l = 0; l < 16 && p0 + l < pairs; l++)
        for (int i = 0; i < 8; i++) cvs[cur ^ 1][p0 + l][i] = w[i][l];
    }
    if (count & 1) memcpy(cvs[cur ^ 1][pairs], cvs[cur][count - 1], 32);
    count = pairs + (count & 1);
    cur ^= 1;
  }
  return ((uint64_t)__builtin_bswap32(cvs[cur][0][0]) << 32) | __builtin_bswap32(cvs[cur][0][1]);
}

typedef struct {
  const uint8_t* arena; const uint64_t* offs; const uint64_t* lens; const uint64_t* sizes;
  uint64_t stride, clen; size_t lo, hi; uint64_t* out; int simd;
} fjob_t;

static void* fast_worker(void* p) {
  fjob_t* j = (fjob_t*)p;
  size_t i = j->lo;
  if (j->simd) {
    for (; i + 16 <= j->hi; i += 16) {
      const uint8_t* ptr[16];
      int uniform = 1;
      uint64_t cl = j->offs ? j->lens[i] : j->clen;
      for (int l = 0; l < 16; l++) {
        ptr[l] = j->offs ? j->arena + j->offs[i + l] : j->arena + (i + l) * j->stride;
        if (j->offs && j->lens[i + l] != cl) uniform = 0;
      }
      if (uniform) cas16(ptr, j->sizes + i, (size_t)cl, j->out + i);
      else
        for (int l = 0; l < 16; l++)
          j->out[i + l] = cas_chunkpar16(ptr[l], (size_t)j->lens[i + l], j->sizes[i + l]);
    }
  }
  for (; i < j->hi; i++) {
    if (j->offs) j->out[i] = orc_cas_key(j->arena + j->offs[i], (size_t)j->lens[i], j->sizes[i]);
    else j->out[i] = orc_cas_key(j->arena + i * j->stride, (size_t)j->clen, j->sizes[i]);
  }
  return NULL;
}

int orc_fast_has_simd(void) {
  __builtin_cpu_init();
  return __builtin_cpu_supports("avx512f");
}

/* Same contract as orc_cas_keys / orc_cas_keys_strided (offs == NULL -> strided). */
void orc_fast_cas_keys(const uint8_t* arena, const uint64_t* offs, const uint64_t* lens,
                       uint64_t stride, uint64_t clen, const uint64_t* sizes, size_t n,
                       uint64_t* out, int threads) {
  int simd = orc_fast_has_simd();
  if (threads < 1) threads = 1;
  size_t groups = (n + 15) / 16;
  if ((size_t)threads > groups) threads = groups ? (int)groups : 1;
  pthread_t* th = calloc((size_t)threads, sizeof *th);
  fjob_t* jobs = calloc((size_t)threads, sizeof *jobs);
  for (int t = 0; t < threads; t++) {
    fjob_t f = {arena, offs, lens, sizes, stride, clen, 0, 0, out, simd};
    f.lo = 16 * (groups * (size_t)t / (size_t)threads);
    f.hi = 16 * (groups * (size_t)(t + 1) / (size_t)threads);
    if (f.hi > n) f.hi = n;
    jobs[t] = f;
    if (threads == 1) fast_worker(&jobs[t]);
    else pthread_create(&th[t], NULL, fast_worker, &jobs[t]);
  }
  if (threads > 1)
    for (int t = 0; t < threads; t++) pthread_join(th[t], NULL);
  free(th); free(jobs);
}

/* Config-1 all-cores baseline with the SIMD hasher: each worker gathers its files
 * (orc_gather_path: the cas.rs offsets) and hashes sampled files 16 at a time with
 * cas16; whole (ragged) files are hashed chunk-parallel (cas_chunkpar16).  keys[i] = 0 and
 * status[i] = -errno for a failed file. */
typedef struct {
  const char* const* paths; const uint64_t* sizes; size_t n; int t, threads, simd;
  uint64_t* keys; int32_t* status;
} fpjob_t;

static void* fast_paths_worker(void* p) {
  fpjob_t* j = (fpjob_t*)p;
  const size_t S = ORC_SAMPLED_CONTENT_LEN, SMALL = ORC_MINIMUM_FILE_SIZE + 1;
  uint8_t* grp = malloc(16 * S);
  uint8_t* one = malloc(SMALL > S ? SMALL : S);
  size_t gi[16];
  uint64_t gs[16], gk[16];
  int ng = 0;
  for (size_t i = (size_t)j->t; i < j->n; i += (size_t)j->threads) {
    const int sampled = j->sizes[i] > ORC_MINIMUM_FILE_SIZE;
    uint8_t* dst = (sampled && j->simd) ? grp + (size_t)ng * S : one;
    int64_t got = orc_gather_path(j->paths[i], j->sizes[i], dst, sampled ? S : SMALL);
    if (got < 0) { j->keys[i] = 0; j->status[i] = (int32_t)got; continue; }
    j->status[i] = 0;
    if (!(sampled && j->simd)) {
      j->keys[i] = j->simd ? cas_chunkpar16(dst, (size_t)got, j->sizes[i]) : orc_cas_key(dst, (size_t)got, j->sizes[i]);
      continue;
    }
    gi[ng] = i; gs[ng] = j->sizes[i]; ng++;
    if (ng == 16) {
      const uint8_t* ptr[16];
      for (int l = 0; l < 16; l++) ptr[l] = grp + (size_t)l * S;
      cas16(ptr, gs, S, gk);
      for (int l = 0; l < 16; l++) j->keys[gi[l]] = gk[l];
      ng = 0;
    }
  }
  for (int l = 0; l < ng; l++) j->keys[gi[l]] = orc_cas_key(grp + (size_t)l * S, S, gs[l]);
  free(grp); free(one);
  return NULL;
}

void orc_fast_generate_cas_keys_paths(const char* const* paths, const uint64_t* sizes, size_t n,
                                      int threads, uint64_t* keys, int32_t* status) {
  const int simd = orc_fast_has_simd();
  if (threads < 1) threads = 1;
  pthread_t* th = calloc((size_t)threads, sizeof *th);
  fpjob_t* jobs = calloc((size_t)threads, sizeof *jobs);
  for (int t = 0; t < threads; t++) {
    jobs[t] = (fpjob_t){paths, sizes, n, t, threads, simd, keys, status};
    if (threads == 1) fast_paths_worker(&jobs[t]);
    else pthread_create(&th[t], NULL, fast_paths_worker, &jobs[t]);
  }
  if (threads > 1)
    for (int t = 0; t < threads; t++) pthread_join(th[t], NULL);
  free(th); free(jobs);
}
