/*
 * oracle.h — CPU restatement of the reference's content-identification path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load this library, and only as the checker / CPU baseline.
 * The product path (spacedrive_amd/, libsd_hip_cas.so) never links or calls it.
 *
 * What it restates (reference = annihilatorrrr/spacedrive @ 2025-01-17):
 *   - BLAKE3 hash mode, as used through the external `blake3` 1.5.0 crate
 *     (Cargo.lock:1127-1139; call sites core/src/object/cas.rs:24-61 and
 *     core/src/object/validation/hash.rs:13-22).  The crate is not vendored in the
 *     reference, so this is a restatement of the published BLAKE3 spec, pinned by the
 *     reference's only in-repo BLAKE3 known answer (derive_key KAT,
 *     crates/crypto/src/keys/hashing.rs:210-213, 323-328), its six Balloon-BLAKE3
 *     KATs (hashing.rs:180-208), by the BLAKE3 team's C implementation (1.8.2, exported
 *     by ROCm's libclang-cpp.so: tests/ext_blake3.py) at every tree shape up to 1 GiB, by
 *     hf_xet's Rust BLAKE3 on trees of 1-128 chunks (keyed mode:
 *     tests/golden/make_xet_vectors.py), and by independent tree formulations that must
 *     agree (incremental CV stack, recursive left-balanced, level-wise, threaded).
 *   - generate_cas_id message layout (core/src/object/cas.rs:10-61).
 *   - file_checksum (core/src/object/validation/hash.rs:11-25).
 *   - Object grouping (core/src/object/file_identifier/mod.rs:98-350), canonical form
 *     and the chunk-of-100 emulation.
 */
#ifndef SD_CAS_ORACLE_H
#define SD_CAS_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- BLAKE3 (spec restatement) ---------------------------------------- */
/* Full BLAKE3 hash, incremental CV-stack formulation. out_len <= 64. */
void orc_blake3(const uint8_t* in, size_t len, uint8_t* out, size_t out_len);
/* Same hash, recursive left-balanced-tree formulation (independent code path). */
void orc_blake3_recursive(const uint8_t* in, size_t len, uint8_t out[32]);
/* Same hash, level-wise pair-and-promote formulation (the GPU validator's shape). */
void orc_blake3_levelwise(const uint8_t* in, size_t len, uint8_t out[32]);
/* blake3::derive_key(context, material) -> 32 bytes. */
void orc_blake3_derive_key(const char* context, const uint8_t* material, size_t len,
                           uint8_t out[32]);
/* blake3::keyed_hash(key, in) -> 32 bytes (formulation 1's tree in KEYED_HASH mode). */
void orc_blake3_keyed(const uint8_t key[32], const uint8_t* in, size_t len, uint8_t out[32]);
/* Same hash, tree-parallel over `threads` pthreads (16 MiB subtrees, then pair-and-promote;
 * SURVEY §8d's "multithreaded tree" CPU mode). */
void orc_blake3_mt(const uint8_t* in, size_t len, int threads, uint8_t out[32]);
/* BLAKE3 of the first `len` bytes of synthetic file `file`'s content stream (the
 * orc_fill_content stream, generated on the fly), tree-parallel. */
void orc_stream_blake3_mt(uint64_t seed, uint64_t file, uint64_t len, int threads, uint8_t out[32]);
/* BLAKE3 over a stream of pieces (== Hasher::update per piece). */
void orc_blake3_pieces(const uint8_t* const* pieces, const size_t* lens, size_t n,
                       uint8_t out[32]);

/* Balloon hashing over BLAKE3 (balloon_ref.c): the reference's password-hash KATs,
 * crates/crypto/src/keys/hashing.rs:180-208 — the multi-block streamed inputs that pin BLAKE3
 * inside a chunk.  secret_len 0 = no secret.  Returns 0, or -1 on bad sizes / no memory. */
int orc_balloon_blake3(const uint8_t* pwd, size_t pwd_len, const uint8_t* salt, size_t salt_len,
                       const uint8_t* secret, size_t secret_len, uint64_t s_cost, uint64_t t_cost,
                       uint8_t out[32]);

/* ---- cas_id (core/src/object/cas.rs) ------------------------------------ */
#define ORC_SAMPLE_COUNT 4ull
#define ORC_SAMPLE_SIZE (1024ull * 10)
#define ORC_HEADER_OR_FOOTER_SIZE (1024ull * 8)
#define ORC_MINIMUM_FILE_SIZE (1024ull * 100)
#define ORC_SAMPLED_CONTENT_LEN (2 * ORC_HEADER_OR_FOOTER_SIZE + ORC_SAMPLE_COUNT * ORC_SAMPLE_SIZE)

/* Byte offsets read by the sampled path for a file of `size` (> MINIMUM_FILE_SIZE):
 * 6 (offset, length) pairs: header, 4 samples, footer. cas.rs:35-58. */
void orc_sample_plan(uint64_t size, uint64_t offs[6], uint64_t lens[6]);
/* Gather the cas content of an in-memory file image (whole file if size<=100 KiB,
 * else the 57,344 sampled bytes). Returns the content length written to out. */
size_t orc_gather_image(const uint8_t* file, uint64_t size, uint8_t* out);
/* Gather from a path with pread, following cas.rs:27-58. Returns content length,
 * or -errno on I/O error (-EIO for a short read == tokio UnexpectedEof). */
int64_t orc_gather_path(const char* path, uint64_t size, uint8_t* out, size_t out_cap);
/* key = big-endian u64 of BLAKE3(le64(size) || content)[0..8]. */
uint64_t orc_cas_key(const uint8_t* content, size_t content_len, uint64_t size);
/* keys for n files packed in one arena */
void orc_cas_keys(const uint8_t* arena, const uint64_t* offs, const uint64_t* lens,
                  const uint64_t* sizes, size_t n, uint64_t* out_keys, int threads);
/* uniform-stride sampled batch (content_len == 57,344 for every file) */
void orc_cas_keys_strided(const uint8_t* arena, uint64_t stride, uint64_t content_len,
                          const uint64_t* sizes, size_t n, uint64_t* out_keys, int threads);
/* 16 lowercase hex chars + NUL */
void orc_key_hex(uint64_t key, char out[17]);
/* generate_cas_id(path, size) -> 0 and out[17], or -errno */
int orc_generate_cas_id(const char* path, uint64_t size, char out[17]);
void orc_generate_cas_keys_paths(const char* const* paths, const uint64_t* sizes, size_t n,
                                 int threads, uint64_t* keys, int32_t* status);
void orc_fast_generate_cas_keys_paths(const char* const* paths, const uint64_t* sizes, size_t n,
                                      int threads, uint64_t* keys, int32_t* status);
/* file_checksum(path) -> 0 and 64-hex, or -errno (hash.rs:11-25): the reference loop
 * literally — 1 MiB reads into one hasher until the first read shorter than 1 MiB */
int orc_file_checksum(const char* path, char out[65]);
/* same digest for a regular file that does not change while read, tree-parallel */
int orc_file_checksum_mt(const char* path, int threads, char out[65]);

/* ---- grouping (core/src/object/file_identifier/mod.rs:98-350) ---------- */
/* canonical: rep[i] = min{ j : key[j] == key[i] }; returns #objects (distinct keys). */
uint64_t orc_group_canonical(const uint64_t* keys, size_t n, uint32_t* rep);
/* chunk-of-`chunk` emulation with HashMap order := ascending idx:
 * rep[i] = i if first chunk containing key[i] is i's own chunk, else canonical rep.
 * created/linked are the summed per-step counts identifier_job_step returns. */
void orc_group_chunked(const uint64_t* keys, size_t n, size_t chunk, uint32_t* rep,
                       uint64_t* created, uint64_t* linked);

/* ---- SIMD CPU baseline (cas_fast.c): 16 files per AVX-512 lane group ---- */
int orc_fast_has_simd(void);
/* offs == NULL -> strided layout (stride, clen); else packed (offs, lens). */
void orc_fast_cas_keys(const uint8_t* arena, const uint64_t* offs, const uint64_t* lens,
                       uint64_t stride, uint64_t clen, const uint64_t* sizes, size_t n,
                       uint64_t* out, int threads);

/* ---- synthetic inputs (shared with the device generator) ---------------- */
uint64_t orc_mix64(uint64_t z);
uint64_t orc_file_key(uint64_t seed, uint64_t file);
void orc_fill_content(uint64_t seed, uint64_t file, uint8_t* out, size_t len);
/* bytes [off, off+len) of the same stream */
void orc_fill_content_range(uint64_t seed, uint64_t file, uint64_t off, uint8_t* out, size_t len);
/* duplicate chain root and synthetic size (kind 0 = sampled, 1 = whole-file) */
uint64_t orc_synth_root(uint64_t seed, uint64_t f, uint32_t dup_permille);
uint64_t orc_synth_size(uint64_t seed, uint64_t root, uint32_t kind);

#ifdef __cplusplus
}
#endif
#endif
