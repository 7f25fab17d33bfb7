/*
 * blake3_ref.c — portable BLAKE3 restated from the published spec.
 *
 * TEST INFRASTRUCTURE ONLY (see oracle.h).  The reference uses the external
 * `blake3` 1.5.0 crate (Cargo.lock:1127-1139), which is not vendored under
 * /root/reference; its algorithm is restated here:
 *   IV = SHA-256 IV; 7 rounds; message permutation [2,6,3,10,7,0,4,13,1,11,12,5,9,14,15,8];
 *   G rotations 16/12/8/7; flags CHUNK_START 1, CHUNK_END 2, PARENT 4, ROOT 8,
 *   KEYED_HASH 16, DERIVE_KEY_CONTEXT 32, DERIVE_KEY_MATERIAL 64; 1024-B chunks of
 *   64-B blocks; left-balanced binary tree.
 * Three independent tree drivers are provided (incremental CV stack, recursive
 * left-balanced split, level-wise pair-and-promote); tests require they agree.
 */
#define _GNU_SOURCE
#include <errno.h>
#include <fcntl.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>
#include <unistd.h>

#include "oracle.h"

#define B3_CHUNK_START 1u
#define B3_CHUNK_END 2u
#define B3_PARENT 4u
#define B3_ROOT 8u
#define B3_KEYED 16u
#define B3_DK_CONTEXT 32u
#define B3_DK_MATERIAL 64u
#define B3_BLOCK 64u
#define B3_CHUNK 1024u

static const uint32_t IV[8] = {0x6A09E667u, 0xBB67AE85u, 0x3C6EF372u, 0xA54FF53Au,
                               0x510E527Fu, 0x9B05688Cu, 0x1F83D9ABu, 0x5BE0CD19u};
static const uint8_t PERM[16] = {2, 6, 3, 10, 7, 0, 4, 13, 1, 11, 12, 5, 9, 14, 15, 8};

static inline uint32_t rotr(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }
static inline uint32_t ld32(const uint8_t* p) {
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}
static inline void st32(uint8_t* p, uint32_t v) {
  p[0] = (uint8_t)v; p[1] = (uint8_t)(v >> 8); p[2] = (uint8_t)(v >> 16); p[3] = (uint8_t)(v >> 24);
}

static inline void g(uint32_t* s, int a, int b, int c, int d, uint32_t x, uint32_t y) {
  s[a] = s[a] + s[b] + x; s[d] = rotr(s[d] ^ s[a], 16);
  s[c] = s[c] + s[d];     s[b] = rotr(s[b] ^ s[c], 12);
  s[a] = s[a] + s[b] + y; s[d] = rotr(s[d] ^ s[a], 8);
  s[c] = s[c] + s[d];     s[b] = rotr(s[b] ^ s[c], 7);
}

/* full 16-word compression output */
static void compress(const uint32_t cv[8], const uint8_t block[64], uint32_t blen,
                     uint64_t counter, uint32_t flags, uint32_t out[16]) {
  uint32_t m[16], s[16], t[16];
  for (int i = 0; i < 16; i++) m[i] = ld32(block + 4 * i);
  for (int i = 0; i < 8; i++) s[i] = cv[i];
  for (int i = 0; i < 4; i++) s[8 + i] = IV[i];
  s[12] = (uint32_t)counter; s[13] = (uint32_t)(counter >> 32); s[14] = blen; s[15] = flags;
  for (int r = 0; r < 7; r++) {
    g(s, 0, 4, 8, 12, m[0], m[1]);   g(s, 1, 5, 9, 13, m[2], m[3]);
    g(s, 2, 6, 10, 14, m[4], m[5]);  g(s, 3, 7, 11, 15, m[6], m[7]);
    g(s, 0, 5, 10, 15, m[8], m[9]);  g(s, 1, 6, 11, 12, m[10], m[11]);
    g(s, 2, 7, 8, 13, m[12], m[13]); g(s, 3, 4, 9, 14, m[14], m[15]);
    if (r < 6) {
      for (int i = 0; i < 16; i++) t[i] = m[PERM[i]];
      memcpy(m, t, sizeof m);
    }
  }
  for (int i = 0; i < 8; i++) { out[i] = s[i] ^ s[i + 8]; out[i + 8] = s[i + 8] ^ cv[i]; }
}

/* An "output": the inputs of a not-yet-finalized compression (root needs ROOT flag). */
typedef struct { uint32_t cv[8]; uint8_t block[64]; uint32_t blen; uint64_t counter; uint32_t flags; } b3_output;

static void output_cv(const b3_output* o, uint32_t cv[8]) {
  uint32_t w[16];
  compress(o->cv, o->block, o->blen, o->counter, o->flags, w);
  memcpy(cv, w, 32);
}
static void output_root(const b3_output* o, uint8_t* out, size_t out_len) {
  /* only out_len <= 64 (one output block) is ever needed on this path */
  uint32_t w[16];
  uint8_t buf[64];
  compress(o->cv, o->block, o->blen, 0, o->flags | B3_ROOT, w);
  for (int i = 0; i < 16; i++) st32(buf + 4 * i, w[i]);
  memcpy(out, buf, out_len > 64 ? 64 : out_len);
}

/* chunk: bytes [0, len) with len <= 1024 (len may be 0 only for the empty input) */
static b3_output chunk_output(const uint32_t key[8], const uint8_t* p, size_t len,
                              uint64_t counter, uint32_t base_flags) {
  b3_output o;
  uint32_t cv[8];
  memcpy(cv, key, 32);
  size_t nblocks = len == 0 ? 1 : (len + 63) / 64;
  for (size_t b = 0; b < nblocks; b++) {
    size_t off = b * 64, bl = len - off < 64 ? len - off : 64;
    if (len == 0) bl = 0;
    uint32_t flags = base_flags | (b == 0 ? B3_CHUNK_START : 0) | (b + 1 == nblocks ? B3_CHUNK_END : 0);
    uint8_t blk[64] = {0};
    if (bl) memcpy(blk, p + off, bl);
    if (b + 1 == nblocks) {
      memcpy(o.cv, cv, 32); memcpy(o.block, blk, 64);
      o.blen = (uint32_t)bl; o.counter = counter; o.flags = flags;
    } else {
      uint32_t w[16];
      compress(cv, blk, 64, counter, flags, w);
      memcpy(cv, w, 32);
    }
  }
  return o;
}

static b3_output parent_output(const uint32_t key[8], const uint32_t l[8], const uint32_t r[8],
                               uint32_t base_flags) {
  b3_output o;
  memcpy(o.cv, key, 32);
  for (int i = 0; i < 8; i++) { st32(o.block + 4 * i, l[i]); st32(o.block + 32 + 4 * i, r[i]); }
  o.blen = 64; o.counter = 0; o.flags = base_flags | B3_PARENT;
  return o;
}

/* ---- formulation 1: incremental CV stack (merge when chunk count has trailing zeros) */
static void hash_stack(const uint32_t key[8], uint32_t flags, const uint8_t* in, size_t len,
                       uint8_t* out, size_t out_len) {
  uint32_t stack[64][8];
  int sp = 0;
  uint64_t nchunks = len == 0 ? 1 : (len + B3_CHUNK - 1) / B3_CHUNK;
  for (uint64_t c = 0; c + 1 < nchunks; c++) {
    b3_output o = chunk_output(key, in + c * B3_CHUNK, B3_CHUNK, c, flags);
    uint32_t cv[8];
    output_cv(&o, cv);
    uint64_t total = c + 1;
    while ((total & 1) == 0) {
      b3_output p = parent_output(key, stack[--sp], cv, flags);
      output_cv(&p, cv);
      total >>= 1;
    }
    memcpy(stack[sp++], cv, 32);
  }
  uint64_t last = nchunks - 1;
  b3_output o = chunk_output(key, in + last * B3_CHUNK, len - last * B3_CHUNK, last, flags);
  while (sp > 0) {
    uint32_t cv[8];
    output_cv(&o, cv);
    o = parent_output(key, stack[--sp], cv, flags);
  }
  output_root(&o, out, out_len);
}

void orc_blake3(const uint8_t* in, size_t len, uint8_t* out, size_t out_len) {
  hash_stack(IV, 0, in, len, out, out_len);
}

/* blake3::keyed_hash(key, in) (KEYED_HASH mode: the key replaces IV in every chunk and
 * parent compression, flag 16 on all of them).  The tree is formulation 1's; this mode is
 * how an independent BLAKE3 in the image (hf_xet's, tests/golden/make_xet_vectors.py) pins
 * that tree on messages of up to 128 chunks. */
void orc_blake3_keyed(const uint8_t key[32], const uint8_t* in, size_t len, uint8_t out[32]) {
  uint32_t k[8];
  for (int i = 0; i < 8; i++) k[i] = ld32(key + 4 * i);
  hash_stack(k, B3_KEYED, in, len, out, 32);
}

/* ---- formulation 2: recursive left-balanced split ------------------------ */
static uint64_t largest_pow2_below(uint64_t n) { /* largest power of two strictly < n, n >= 2 */
  uint64_t p = 1;
  while (p * 2 < n) p *= 2;
  return p;
}
static b3_output rec_output(const uint8_t* in, size_t len, uint64_t chunk0) {
  if (len <= B3_CHUNK) return chunk_output(IV, in, len, chunk0, 0);
  uint64_t nchunks = (len + B3_CHUNK - 1) / B3_CHUNK;
  uint64_t left_chunks = largest_pow2_below(nchunks);
  size_t left_len = (size_t)(left_chunks * B3_CHUNK);
  b3_output lo = rec_output(in, left_len, chunk0);
  b3_output ro = rec_output(in + left_len, len - left_len, chunk0 + left_chunks);
  uint32_t l[8], r[8];
  output_cv(&lo, l); output_cv(&ro, r);
  return parent_output(IV, l, r, 0);
}
void orc_blake3_recursive(const uint8_t* in, size_t len, uint8_t out[32]) {
  b3_output o = rec_output(in, len, 0);
  output_root(&o, out, 32);
}

/* ---- formulation 3: level-wise pair-and-promote -------------------------- */
void orc_blake3_levelwise(const uint8_t* in, size_t len, uint8_t out[32]) {
  uint64_t n = len == 0 ? 1 : (len + B3_CHUNK - 1) / B3_CHUNK;
  if (n == 1) { b3_output o = chunk_output(IV, in, len, 0, 0); output_root(&o, out, 32); return; }
  uint32_t (*cv)[8] = malloc(n * 32);
  for (uint64_t c = 0; c < n; c++) {
    size_t cl = (c + 1 < n) ? B3_CHUNK : len - c * B3_CHUNK;
    b3_output o = chunk_output(IV, in + c * B3_CHUNK, cl, c, 0);
    output_cv(&o, cv[c]);
  }
  while (n > 2) {
    uint64_t m = 0;
    for (uint64_t i = 0; i + 1 < n; i += 2) {
      b3_output p = parent_output(IV, cv[i], cv[i + 1], 0);
      output_cv(&p, cv[m++]);
    }
    if (n & 1) memcpy(cv[m++], cv[n - 1], 32);
    n = m;
  }
  b3_output root = parent_output(IV, cv[0], cv[1], 0);
  output_root(&root, out, 32);
  free(cv);
}

/* ---- derive_key (pins compression + flags against the crypto crate KAT) --- */
void orc_blake3_derive_key(const char* context, const uint8_t* material, size_t len,
                           uint8_t out[32]) {
  uint8_t ck[32];
  uint32_t key[8];
  hash_stack(IV, B3_DK_CONTEXT, (const uint8_t*)context, strlen(context), ck, 32);
  for (int i = 0; i < 8; i++) key[i] = ld32(ck + 4 * i);
  hash_stack(key, B3_DK_MATERIAL, material, len, out, 32);
}

void orc_blake3_pieces(const uint8_t* const* pieces, const size_t* lens, size_t n,
                       uint8_t out[32]) {
  size_t total = 0;
  for (size_t i = 0; i < n; i++) total += lens[i];
  uint8_t* buf = malloc(total ? total : 1);
  size_t off = 0;
  for (size_t i = 0; i < n; i++) { memcpy(buf + off, pieces[i], lens[i]); off += lens[i]; }
  orc_blake3(buf, total, out, 32);
  free(buf);
}

/* ---- tree-parallel driver (SURVEY §8d "multithreaded tree"; test infrastructure) ------
 * The left-balanced tree over N chunks, level-wise: node i of level k covers chunks
 * [i*2^k, min((i+1)*2^k, N)).  Threads compute the level-K nodes (complete subtrees of
 * 2^K chunks, the last one possibly partial) independently; their CVs are then merged by
 * pair-and-promote with ROOT on the final parent — the same tree as formulations 1-3. */
#include <pthread.h>

/* non-root CV of the subtree over in[0, len) (len > 0) whose first chunk is chunk0 */
static void subtree_cv(const uint8_t* in, size_t len, uint64_t chunk0, uint32_t cv[8]) {
  uint32_t stack[64][8];
  int sp = 0;
  const uint64_t nchunks = (len + B3_CHUNK - 1) / B3_CHUNK;
  for (uint64_t c = 0; c < nchunks; c++) {
    const size_t cl = len - c * B3_CHUNK < B3_CHUNK ? len - c * B3_CHUNK : B3_CHUNK;
    b3_output o = chunk_output(IV, in + c * B3_CHUNK, cl, chunk0 + c, 0);
    uint32_t x[8];
    output_cv(&o, x);
    for (uint64_t total = c + 1; (total & 1) == 0; total >>= 1) {
      b3_output p = parent_output(IV, stack[--sp], x, 0);
      output_cv(&p, x);
    }
    memcpy(stack[sp++], x, 32);
  }
  uint32_t cur[8];
  memcpy(cur, stack[--sp], 32);
  while (sp > 0) {
    b3_output p = parent_output(IV, stack[--sp], cur, 0);
    output_cv(&p, cur);
  }
  memcpy(cv, cur, 32);
}

/* source of the message bytes [off, off+len): returns a pointer to them (in `scratch`, of
 * at least len bytes, or in place) */
typedef const uint8_t* (*b3_src_fn)(void* ctx, uint64_t off, size_t len, uint8_t* scratch);

#define MT_SUB_CHUNKS (1u << 14) /* 16 MiB subtrees */

typedef struct {
  b3_src_fn src; void* ctx; uint64_t len, nsub; uint32_t (*cvs)[8];
  uint64_t next; int err;
} mt_job;

static void* mt_worker(void* p) {
  mt_job* j = (mt_job*)p;
  const size_t sub_bytes = (size_t)MT_SUB_CHUNKS * B3_CHUNK;
  uint8_t* scratch = malloc(sub_bytes);
  if (!scratch) { __atomic_store_n(&j->err, 1, __ATOMIC_RELAXED); return NULL; }
  for (;;) {
    const uint64_t s = __atomic_fetch_add(&j->next, 1, __ATOMIC_RELAXED);
    if (s >= j->nsub) break;
    const uint64_t off = s * sub_bytes;
    const size_t n = (size_t)(j->len - off < sub_bytes ? j->len - off : sub_bytes);
    const uint8_t* d = j->src(j->ctx, off, n, scratch);
    if (!d) { __atomic_store_n(&j->err, 1, __ATOMIC_RELAXED); break; }
    subtree_cv(d, n, s * MT_SUB_CHUNKS, j->cvs[s]);
  }
  free(scratch);
  return NULL;
}

static int blake3_mt_src(b3_src_fn src, void* ctx, uint64_t len, int threads, uint8_t out[32]) {
  const uint64_t sub_bytes = (uint64_t)MT_SUB_CHUNKS * B3_CHUNK;
  if (len <= sub_bytes) { /* one subtree holds the root */
    uint8_t* scratch = malloc(len ? len : 1);
    const uint8_t* d = src(ctx, 0, (size_t)len, scratch);
    if (d) orc_blake3(d, (size_t)len, out, 32);
    free(scratch);
    return d ? 0 : -1;
  }
  mt_job j = {src, ctx, len, (len + sub_bytes - 1) / sub_bytes, NULL, 0, 0};
  j.cvs = malloc(j.nsub * 32);
  if (threads < 1) threads = 1;
  if ((uint64_t)threads > j.nsub) threads = (int)j.nsub;
  pthread_t th[256];
  if (threads > 256) threads = 256;
  for (int t = 1; t < threads; t++) pthread_create(&th[t], NULL, mt_worker, &j);
  mt_worker(&j);
  for (int t = 1; t < threads; t++) pthread_join(th[t], NULL);
  if (j.err) { free(j.cvs); return -1; }
  uint64_t n = j.nsub;
  while (n > 2) { /* pair-and-promote over the level-K nodes */
    uint64_t m = 0;
    for (uint64_t i = 0; i + 1 < n; i += 2) {
      b3_output p = parent_output(IV, j.cvs[i], j.cvs[i + 1], 0);
      output_cv(&p, j.cvs[m++]);
    }
    if (n & 1) memcpy(j.cvs[m++], j.cvs[n - 1], 32);
    n = m;
  }
  b3_output root = parent_output(IV, j.cvs[0], j.cvs[1], 0);
  output_root(&root, out, 32);
  free(j.cvs);
  return 0;
}

static const uint8_t* src_mem(void* ctx, uint64_t off, size_t len, uint8_t* scratch) {
  (void)len; (void)scratch;
  return (const uint8_t*)ctx + off;
}

void orc_blake3_mt(const uint8_t* in, size_t len, int threads, uint8_t out[32]) {
  (void)blake3_mt_src(src_mem, (void*)in, len, threads, out);
}

typedef struct { uint64_t seed, file; } stream_ctx;
static const uint8_t* src_stream(void* ctx, uint64_t off, size_t len, uint8_t* scratch) {
  const stream_ctx* s = (const stream_ctx*)ctx;
  orc_fill_content_range(s->seed, s->file, off, scratch, len);
  return scratch;
}

void orc_stream_blake3_mt(uint64_t seed, uint64_t file, uint64_t len, int threads, uint8_t out[32]) {
  stream_ctx s = {seed, file};
  (void)blake3_mt_src(src_stream, &s, len, threads, out);
}

static const uint8_t* src_fd(void* ctx, uint64_t off, size_t len, uint8_t* scratch) {
  const int fd = *(const int*)ctx;
  size_t got = 0;
  while (got < len) {
    ssize_t r = pread(fd, scratch + got, len - got, (off_t)(off + got));
    if (r < 0 && errno == EINTR) continue;
    if (r <= 0) return NULL;
    got += (size_t)r;
  }
  return scratch;
}

/* file_checksum of a regular file that does not change while it is read: the digest of its
 * st_size bytes, subtrees read with pread by `threads` workers */
int orc_file_checksum_mt(const char* path, int threads, char out[65]) {
  int fd = open(path, O_RDONLY | O_CLOEXEC);
  if (fd < 0) return -errno;
  struct stat st;
  if (fstat(fd, &st) != 0) { int e = -errno; close(fd); return e; }
  uint8_t h[32];
  int rc = blake3_mt_src(src_fd, &fd, (uint64_t)st.st_size, threads, h);
  close(fd);
  if (rc) return -EIO;
  static const char* hx = "0123456789abcdef";
  for (int i = 0; i < 32; i++) { out[2 * i] = hx[h[i] >> 4]; out[2 * i + 1] = hx[h[i] & 15]; }
  out[64] = 0;
  return 0;
}
