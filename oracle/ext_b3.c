/*
 * ext_b3.c — the reference's per-file hashing sequence run by the BLAKE3 team's own C
 * implementation (test / CPU-baseline infrastructure; see oracle.h for who may load it).
 *
 * cas.rs:23-62 hashes a file as Hasher::new(); update(le64(size)); update(content);
 * finalize().  The `blake3` crate it calls (1.5.0, Cargo.lock:1127-1139) is not vendored, but
 * the BLAKE3 team's C implementation (1.8.2, portable + SSE4.1/AVX2/AVX-512 kernels that the
 * crate's own SIMD back ends mirror) ships in this image inside LLVM, exported by ROCm's
 * libclang-cpp.so as llvm_blake3_hasher_*.  This file dlopens it (no link-time dependency;
 * RTLD_LOCAL) and runs that exact sequence per file, files statically partitioned over
 * pthreads — the rayon-style all-cores baseline BASELINE.json names, with the library the
 * crate's authors wrote in place of the crate.  Keys: big-endian u64 of digest[0..8].
 */
#define _GNU_SOURCE
#include <dlfcn.h>
#include <errno.h>
#include <fcntl.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include "oracle.h" /* orc_gather_path: cas.rs's reads (liboracle_cas.so) */

#define EXT_B3_LIB "/opt/rocm/lib/llvm/lib/libclang-cpp.so"
#define HASHER_BYTES 4096 /* sizeof(llvm_blake3_hasher) is 1,912 */

typedef void (*init_fn)(void*);
typedef void (*update_fn)(void*, const void*, size_t);
typedef void (*finalize_fn)(const void*, uint8_t*, size_t);
typedef const char* (*version_fn)(void);

static init_fn b3_init;
static update_fn b3_update;
static finalize_fn b3_finalize;
static version_fn b3_version;

/* 0 = loaded; -1 = library or symbols missing */
int ext_b3_load(void) {
  if (b3_init) return 0;
  void* h = dlopen(EXT_B3_LIB, RTLD_NOW | RTLD_LOCAL);
  if (!h) return -1;
  b3_init = (init_fn)dlsym(h, "llvm_blake3_hasher_init");
  b3_update = (update_fn)dlsym(h, "llvm_blake3_hasher_update");
  b3_finalize = (finalize_fn)dlsym(h, "llvm_blake3_hasher_finalize");
  b3_version = (version_fn)dlsym(h, "llvm_blake3_version");
  if (!b3_init || !b3_update || !b3_finalize || !b3_version) {
    b3_init = NULL;
    return -1;
  }
  return 0;
}

const char* ext_b3_version(void) { return ext_b3_load() ? "" : b3_version(); }

static uint64_t cas_key(const uint8_t* content, size_t clen, uint64_t size) {
  _Alignas(64) uint8_t hasher[HASHER_BYTES];
  uint8_t le[8], out[32];
  for (int i = 0; i < 8; i++) le[i] = (uint8_t)(size >> (8 * i));
  b3_init(hasher);
  b3_update(hasher, le, 8);
  b3_update(hasher, content, clen);
  b3_finalize(hasher, out, 32);
  uint64_t k = 0;
  for (int i = 0; i < 8; i++) k = (k << 8) | out[i];
  return k;
}

typedef struct {
  const uint8_t* arena;
  uint64_t stride, clen;
  const uint64_t* sizes;
  uint64_t* keys;
  size_t lo, hi;
} job;

static void* worker(void* p) {
  job* j = (job*)p;
  for (size_t i = j->lo; i < j->hi; i++)
    j->keys[i] = cas_key(j->arena + i * j->stride, (size_t)j->clen, j->sizes[i]);
  return NULL;
}

/* keys[i] = cas key of file i: content arena[i*stride, +clen), size sizes[i]; 0 ok, -1 no
 * library, -ENOMEM. */
int ext_b3_cas_keys_strided(const uint8_t* arena, uint64_t stride, uint64_t clen,
                            const uint64_t* sizes, size_t n, uint64_t* keys, int threads) {
  if (ext_b3_load()) return -1;
  if (threads < 1) threads = 1;
  if ((size_t)threads > n) threads = n ? (int)n : 1;
  pthread_t* th = malloc(sizeof(pthread_t) * (size_t)threads);
  job* js = malloc(sizeof(job) * (size_t)threads);
  if (!th || !js) { free(th); free(js); return -ENOMEM; }
  int started[threads];
  for (int t = 0; t < threads; t++) {
    js[t] = (job){arena, stride, clen, sizes, keys, n * (size_t)t / (size_t)threads,
                  n * (size_t)(t + 1) / (size_t)threads};
    started[t] = t && pthread_create(&th[t], NULL, worker, &js[t]) == 0;
  }
  worker(&js[0]);
  for (int t = 1; t < threads; t++) {
    if (started[t]) pthread_join(th[t], NULL);
    else worker(&js[t]);  /* a thread that could not start: its share on this thread */
  }
  free(th);
  free(js);
  return 0;
}

/* ---- the paths forms: the reference's reads, the C library's hashing ------------------ */

/* hash.rs:11-25 streamed: one hasher, read(1 MiB) and update with what was read, stop at
 * the first read shorter than 1 MiB.  out: 64 hex + NUL.  0 ok, -errno, -1000 no library. */
int ext_b3_file_checksum(const char* path, char out[65]) {
  enum { BLOCK_LEN = 1 << 20 };
  if (ext_b3_load()) return -1000;
  int fd = open(path, O_RDONLY | O_CLOEXEC);
  if (fd < 0) return -errno;
  uint8_t* buf = malloc(BLOCK_LEN);
  if (!buf) { close(fd); return -ENOMEM; }
  _Alignas(64) uint8_t hasher[HASHER_BYTES];
  b3_init(hasher);
  for (;;) {
    ssize_t r;
    do { r = read(fd, buf, BLOCK_LEN); } while (r < 0 && errno == EINTR);
    if (r < 0) { int e = -errno; free(buf); close(fd); return e; }
    b3_update(hasher, buf, (size_t)r);
    if (r != BLOCK_LEN) break;
  }
  close(fd);
  free(buf);
  uint8_t h[32];
  b3_finalize(hasher, h, 32);
  static const char* hx = "0123456789abcdef";
  for (int i = 0; i < 32; i++) { out[2 * i] = hx[h[i] >> 4]; out[2 * i + 1] = hx[h[i] & 15]; }
  out[64] = 0;
  return 0;
}

typedef struct {
  const char* const* paths; const uint64_t* sizes; size_t n; int t, threads;
  char* hex; uint64_t* keys; int32_t* status;
} pjob;

static void* sums_worker(void* p) {
  pjob* j = (pjob*)p;
  for (size_t i = (size_t)j->t; i < j->n; i += (size_t)j->threads)
    j->status[i] = ext_b3_file_checksum(j->paths[i], j->hex + 65 * i);
  return NULL;
}

static void* keys_worker(void* p) {
  pjob* j = (pjob*)p;
  const size_t cap = ORC_MINIMUM_FILE_SIZE + 1 > ORC_SAMPLED_CONTENT_LEN ? ORC_MINIMUM_FILE_SIZE + 1
                                                                         : ORC_SAMPLED_CONTENT_LEN;
  uint8_t* buf = malloc(cap);
  for (size_t i = (size_t)j->t; i < j->n; i += (size_t)j->threads) {
    if (!buf) { j->keys[i] = 0; j->status[i] = -ENOMEM; continue; }
    const int64_t got = orc_gather_path(j->paths[i], j->sizes[i], buf, cap);
    if (got < 0) { j->keys[i] = 0; j->status[i] = (int32_t)got; continue; }
    j->keys[i] = cas_key(buf, (size_t)got, j->sizes[i]);
    j->status[i] = 0;
  }
  free(buf);
  return NULL;
}

static int run_paths(pjob proto, void* (*fn)(void*)) {
  if (ext_b3_load()) return -1;
  int threads = proto.threads < 1 ? 1 : proto.threads;
  pthread_t* th = calloc((size_t)threads, sizeof *th);
  pjob* js = calloc((size_t)threads, sizeof *js);
  if (!th || !js) { free(th); free(js); return -ENOMEM; }
  int started[threads > 0 ? threads : 1];
  for (int t = 0; t < threads; t++) {
    js[t] = proto;
    js[t].t = t;
    js[t].threads = threads;
    started[t] = t && pthread_create(&th[t], NULL, fn, &js[t]) == 0;
  }
  fn(&js[0]);
  for (int t = 1; t < threads; t++) {
    if (started[t]) pthread_join(th[t], NULL);
    else fn(&js[t]);  /* a thread that could not start: its share on this thread */
  }
  free(th);
  free(js);
  return 0;
}

/* The validator over many files, files interleaved over `threads` pthreads (each file one
 * hash.rs call).  hex: n x 65 bytes; status[i] 0 or -errno. */
int ext_b3_file_checksums(const char* const* paths, size_t n, int threads, char* hex, int32_t* status) {
  pjob proto = {paths, NULL, n, 0, threads, hex, NULL, status};
  return run_paths(proto, sums_worker);
}

/* cas.rs:23-62 per path: the reference's reads (orc_gather_path: whole file at or below
 * 100 KiB, else header / 4 samples / footer at the cas.rs offsets), then Hasher::new,
 * update(le64(size)), update(content), finalize through the C library. */
int ext_b3_cas_keys_paths(const char* const* paths, const uint64_t* sizes, size_t n, int threads,
                          uint64_t* keys, int32_t* status) {
  pjob proto = {paths, sizes, n, 0, threads, NULL, keys, status};
  return run_paths(proto, keys_worker);
}
