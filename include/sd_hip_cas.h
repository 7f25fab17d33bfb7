/*
 * sd_hip_cas.h — C ABI of the MI355X (gfx950) content-identification engine.
 *
 * Drop-in boundary for the north-star path of annihilatorrrr/spacedrive:
 *   generate_cas_id   core/src/object/cas.rs:23-62
 *   (its batch caller) core/src/object/file_identifier/mod.rs:78-86, 98-350
 *   file_checksum     core/src/object/validation/hash.rs:11-25
 * Plain C: pointers + sizes, no C++ or torch types.  The Rust-side binding
 * (`sd-hip-cas` crate, extern "C" block + safe `generate_cas_ids`) is shown in
 * INTEGRATION.md.
 *
 * Conventions
 *   - Every function returns an int status: SD_CAS_OK (0) or a negative SD_CAS_E*.
 *     The message of the last failure on a context is sd_cas_last_error(ctx);
 *     sd_cas_last_error(NULL) says why this thread's last sd_cas_ctx_create failed.
 *   - A "cas key" is the big-endian u64 of BLAKE3(le64(size) || content)[0..8]:
 *     sd_cas_key_to_hex(key) is exactly the 16-char cas_id String of cas.rs:61, and
 *     numeric key order equals the string order of cas_ids.
 *   - "content" is what generate_cas_id feeds after the size prefix: the whole file
 *     when size <= SD_CAS_MINIMUM_FILE_SIZE (cas.rs:27-29), otherwise the 57,344
 *     gathered bytes header || 4 samples || footer (cas.rs:31-58).
 *   - *_dev functions take device pointers already resident in HBM and a hipStream_t
 *     passed as void* (NULL = the HIP null/default stream, as in HIP; pass
 *     sd_cas_ctx_stream(ctx) for the context's own stream); they enqueue and return
 *     without synchronising unless stated.  Host-buffer functions are blocking and run
 *     on the context's streams.
 *   - Stream ordering is the caller's for its own buffers: a device buffer the caller
 *     initialises (a zeroed flag or counter, a prefilled output) must be written on the
 *     stream passed to the *_dev call, or be complete (event / synchronize) before the
 *     call — the library orders its work on that stream and its internal side streams,
 *     not against other streams.  E.g. torch.zeros(...) runs on torch's current stream: pass
 *     that stream, or synchronise after the fill.
 *   - Contexts are not thread-safe; use one per (thread, device).
 */
#ifndef SD_HIP_CAS_H
#define SD_HIP_CAS_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SD_CAS_ABI_VERSION 1

/* core/src/object/cas.rs:10-15 */
#define SD_CAS_SAMPLE_COUNT 4u
#define SD_CAS_SAMPLE_SIZE (1024u * 10u)
#define SD_CAS_HEADER_OR_FOOTER_SIZE (1024u * 8u)
#define SD_CAS_MINIMUM_FILE_SIZE (1024u * 100u)
#define SD_CAS_SAMPLED_CONTENT_LEN (2u * SD_CAS_HEADER_OR_FOOTER_SIZE + SD_CAS_SAMPLE_COUNT * SD_CAS_SAMPLE_SIZE)
/* file_identifier/mod.rs:34 */
#define SD_CAS_CHUNK_SIZE 100u
/* largest content the packed kernel takes (104 BLAKE3 chunks incl. the size prefix) */
#define SD_CAS_MAX_PACKED_CONTENT_LEN (104u * 1024u - 8u)

#define SD_CAS_OK 0
#define SD_CAS_EINVAL (-1)  /* bad argument (null pointer, misaligned, too large) */
#define SD_CAS_EHIP (-2)    /* HIP runtime / kernel launch failure: batch-level */
#define SD_CAS_EIO (-3)     /* file I/O failure (per-file status carries -errno) */
#define SD_CAS_ENOMEM (-4)  /* device or pinned allocation failed */
#define SD_CAS_ENODEV (-5)  /* no gfx950 device at this ordinal */

typedef struct sd_cas_ctx sd_cas_ctx;

int sd_cas_abi_version(void);

/* ---- context / memory --------------------------------------------------------------- */
int sd_cas_ctx_create(int device, sd_cas_ctx** out);
void sd_cas_ctx_destroy(sd_cas_ctx* ctx);
const char* sd_cas_last_error(const sd_cas_ctx* ctx);
/* the context's compute stream (hipStream_t) */
void* sd_cas_ctx_stream(sd_cas_ctx* ctx);
int sd_cas_synchronize(sd_cas_ctx* ctx);
/* Files per full wave of the device (CUs x 4 SIMDs x 64 lanes; 65,536 on MI355X).  K1/K2
 * run one file per lane, so batches that are a multiple of this avoid a partial last
 * wave round (measured: 1,250,000 files 51.2 M files/s vs 1,310,720 files 55.7 M/s). */
size_t sd_cas_batch_quantum(const sd_cas_ctx* ctx);
/* Batches of fewer than `sampled_files` sampled files (sd_cas_hash_sampled_dev/_host) or
 * `packed_files` whole files (sd_cas_hash_packed_dev) are hashed chunk-parallel — a lane
 * per 1 KiB chunk (or per 4+ chunks, sd_cas_set_chunkpar_split), cross-lane tree merge —
 * for latency (~16 + log2(chunks) compression times per file instead of 953); larger
 * batches use one file per lane for throughput.  Both paths give identical keys.
 * 0 = always one file per lane;
 * SD_CAS_THRESHOLD_DEFAULT = the measured crossover (3/4 and 2x the batch quantum). */
#define SD_CAS_THRESHOLD_DEFAULT ((size_t)-1)
void sd_cas_set_latency_threshold(sd_cas_ctx* ctx, size_t sampled_files, size_t packed_files);
/* Shape of the chunk-parallel path: batches of at least `sampled_files` / `packed_files`
 * files pack four files per wave (16 lanes per file, 4+ consecutive chunks per lane, lane
 * subtrees merged across lanes with DPP row shifts), smaller ones take one wave per file
 * (a lane per chunk, lowest latency).  Identical keys either way.  0 = always four per
 * wave; SD_CAS_THRESHOLD_DEFAULT = the measured crossover (sampled: 3/64, whole files:
 * 3/32 of the batch quantum; whole files are then visited by chunk count, one stable radix
 * pass, so the four files of a wave share a chunks-per-lane class). */
void sd_cas_set_chunkpar_split(sd_cas_ctx* ctx, size_t sampled_files, size_t packed_files);
/* Object grouping method (sd_cas_group_dev / sd_cas_group_min_dev): AUTO = the bucket
 * partition + LDS hash tables (K4h/K5h) up to SD_CAS_HASH_GROUP_MAX_KEYS keys per call and
 * the LSD radix sort + runs (K4/K5) above; HASH / SORT force one (HASH fails beyond the
 * limit).  bucket_target = mean keys per hash bucket (0 = the tuned 1,536; >= 16): smaller
 * targets partition deeper — the plans of > 200M keys at small n, for tests.  Results
 * are identical for every setting. */
#define SD_CAS_GROUP_AUTO 0
#define SD_CAS_GROUP_HASH 1
#define SD_CAS_GROUP_SORT 2
#define SD_CAS_HASH_GROUP_MAX_KEYS (1310720000ull) /* 2^19 buckets x 2,500 keys */
int sd_cas_set_group_method(sd_cas_ctx* ctx, int method, uint64_t bucket_target);
/* page-locked host staging for the gather (replaces the per-file Box<[u8]> of cas.rs:32) */
int sd_cas_alloc_pinned(sd_cas_ctx* ctx, size_t bytes, void** out);
int sd_cas_free_pinned(sd_cas_ctx* ctx, void* p);

/* ---- cas_id: host buffers (blocking) --------------------------------------------------
 * Batched generate_cas_id (cas.rs:23) over already-gathered content:
 *   bufs[i] / buf_lens[i] = content of file i, sizes[i] = fs::metadata().len()
 *   (file_identifier/mod.rs:78-79).  out_keys[i] = cas key.
 * Staged through pinned memory and hipMemcpyAsync on a side stream, then hashed.
 * A sampled file (size > SD_CAS_MINIMUM_FILE_SIZE) must have buf_len == 57,344. */
int sd_cas_generate_cas_ids(sd_cas_ctx* ctx, const uint8_t* const* bufs, const uint64_t* buf_lens,
                            const uint64_t* sizes, size_t n, uint64_t* out_keys);

/* The cas part of FileMetadata::new (file_identifier/mod.rs:55-95) over a batch of paths,
 * gathering each file with pread at the cas.rs:27-58 offsets.  sizes[i] = the file's
 * fs::metadata().len() (mod.rs:63,78-79) as the caller just read it, or sizes == NULL: the
 * library takes that metadata itself (stat, following symlinks, like fs::metadata).
 * status[i] / out_keys[i]:
 *   0                    cas key of generate_cas_id(path, size) (cas.rs:23-62);
 *   SD_CAS_STATUS_NO_CAS metadata length 0: no cas_id (mod.rs:78-86), nothing read, key 0;
 *   -errno               metadata, open or read failed (a short read of a sampled file is
 *                        -EIO == tokio's UnexpectedEof), -EISDIR for a directory (the
 *                        reference asserts, mod.rs:67-70); key 0 — the row is dropped from
 *                        its step like mod.rs:125-141 does.
 * A whole file (0 < size <= 100 KiB) is hashed as it is on disk even when its length no
 * longer matches `size` (cas.rs:29 reads the file, not `size` bytes; one longer than the
 * whole-file limit goes through the validator tree).  Returns SD_CAS_OK unless the batch
 * itself failed. */
#define SD_CAS_STATUS_NO_CAS 1
int sd_cas_generate_cas_ids_from_paths(sd_cas_ctx* ctx, const char* const* paths,
                                       const uint64_t* sizes, size_t n, uint64_t* out_keys,
                                       int32_t* status);
/* FileMetadata::new over a batch with the metadata taken by the library (sizes == NULL
 * above) and returned: out_sizes[i] = the fs::metadata().len() the row was decided from
 * (FileMetadata's fs_metadata, mod.rs:48-53,63), 0 for a row whose metadata failed — one stat
 * per path, so the caller's record can never disagree with the status it got. */
int sd_cas_file_metadata_from_paths(sd_cas_ctx* ctx, const char* const* paths, size_t n,
                                    uint64_t* out_keys, int32_t* status, uint64_t* out_sizes);

/* End-to-end sampled path from host memory (BASELINE config 3 "pre-staged in pinned host
 * memory"): n contents of 57,344 B at h_content + i*stride (pin it with
 * sd_cas_alloc_pinned for overlap), sizes and keys in host memory.  Batches of
 * batch_files (0 = sd_cas_batch_quantum) ping-pong between an H2D copy on the side stream and K1 +
 * D2H of the keys on the compute stream.  Blocking. */
int sd_cas_hash_sampled_host(sd_cas_ctx* ctx, const void* h_content, uint64_t stride,
                             const uint64_t* h_sizes, size_t n, uint64_t* h_keys,
                             size_t batch_files);

/* Same over a host ring of ring_files contents reused cyclically: file i's 57,344 B are at
 * h_ring + (i % ring_files) * stride; h_sizes / h_keys hold all n files.  Every file is
 * copied host -> device (the E2E run of BASELINE config 3 over more files than fit in
 * pinned memory).  Blocking. */
int sd_cas_hash_sampled_host_ring(sd_cas_ctx* ctx, const void* h_ring, uint64_t stride,
                                  size_t ring_files, const uint64_t* h_sizes, size_t n,
                                  uint64_t* h_keys, size_t batch_files);

/* 16 lowercase hex chars + NUL: the cas_id String of cas.rs:61 */
void sd_cas_key_to_hex(uint64_t key, char out[17]);

/* ---- cas_id string consumers: thumbnails -----------------------------
 * get_shard_hex (core/src/object/media/thumbnail/shard.rs:10-13): the first 3 chars of the
 * cas_id (4,096 directories "000".."fff") + NUL. */
void sd_cas_shard_hex(uint64_t key, char out[4]);
/* get_thumbnail_path (thumbnail/mod.rs:67-82): PathBuf pushes of
 *   data_dir / "thumbnails" / (library_id | "ephemeral") / shard / cas_id, extension "webp"
 * library_id NULL = ThumbnailKind::Ephemeral, else the library's UUID string
 * (ThumbnailKind::Indexed).  snprintf-like: writes at most cap bytes incl. the NUL and returns
 * the full path length without it (>= cap: truncated); SD_CAS_EINVAL on a NULL data_dir. */
int64_t sd_cas_thumbnail_path(const char* data_dir, const char* library_id, uint64_t key,
                              char* out, size_t cap);
/* get_thumb_key (thumbnail/mod.rs:94-103): the three strings [library_id | "ephemeral",
 * shard, cas_id], each NUL-terminated, back to back in out.  Returns the bytes needed
 * (written only if <= cap). */
int64_t sd_cas_thumb_key(const char* library_id, uint64_t key, char* out, size_t cap);
/* Device batches (async on stream).  keys_to_hex: d_out[16 i .. 16 i + 16) = the cas_id of
 * key i (no NUL; d_out 16-B aligned).  thumbnail_paths: d_out[stride i ..] = prefix ‖ shard ‖
 * '/' ‖ cas_id ‖ ".webp", NUL-padded to stride, where prefix is one kind's directory with its
 * trailing '/' (sd_cas_thumbnail_path's result minus its last 25 chars, <= 1,024 B);
 * stride a multiple of 16, <= 2,048, >= strlen(prefix) + 26. */
int sd_cas_keys_to_hex_dev(sd_cas_ctx* ctx, const uint64_t* d_keys, size_t n, char* d_out,
                           void* stream);
int sd_cas_thumbnail_paths_dev(sd_cas_ctx* ctx, const uint64_t* d_keys, size_t n,
                               const char* prefix, uint32_t stride, char* d_out, void* stream);

/* ---- cas_id: device-resident batches (async on stream) --------------------------------
 * K1 sampled path: n contents of exactly 57,344 B at d_content + i*stride
 * (stride >= 57,344, multiple of 16; d_content 16-B aligned). */
int sd_cas_hash_sampled_dev(sd_cas_ctx* ctx, const void* d_content, uint64_t stride,
                            const uint64_t* d_sizes, size_t n, uint64_t* d_keys, void* stream);

/* K2 packed path: content i at d_arena + d_offs[i] (16-B aligned), d_lens[i] bytes
 * (<= SD_CAS_MAX_PACKED_CONTENT_LEN); the arena must be readable up to the 16-B round-up
 * of every content end and for at least 16 bytes from every content start (an empty
 * content included).  Files are visited longest-first via an on-device length sort
 * (workspace in ctx).  128-B aligned offsets are recommended (what the library's own
 * host packing and synth_small use): a lane's 128-B line pair then maps to one cache
 * line — 16-B packing reads 1.13x the content bytes from HBM and runs ~2.5 % slower. */
int sd_cas_hash_packed_dev(sd_cas_ctx* ctx, const void* d_arena, const uint64_t* d_offs,
                           const uint32_t* d_lens, const uint64_t* d_sizes, size_t n,
                           uint64_t* d_keys, void* stream);

/* ---- Object grouping (file_identifier/mod.rs:98-350) ----------------------------------
 * Canonical: d_rep[i] = min{ j : key[j] == key[i] } (the file whose Object file i links
 * to); *out_objects = number of Objects (= distinct keys).  Blocks until done when
 * out_objects != NULL.  n < 2^32. */
int sd_cas_group_dev(sd_cas_ctx* ctx, const uint64_t* d_keys, size_t n, uint32_t* d_rep,
                     uint64_t* out_objects, void* stream);
/* Hash + group in one chain (a sampled batch of the file identifier: generate_cas_id for
 * every file, then the grouping of mod.rs:98-350): d_keys as sd_cas_hash_sampled_dev, d_rep
 * as sd_cas_group_dev.  K1 partitions its own keys in its epilogue — each (mixed key, file)
 * row goes to a fixed-capacity region of its coarse bucket — so the grouping after it is one
 * bucket-table launch (no key read-back, totals, prefill or scatter pass).  Async unless
 * out_objects != NULL.  d_overflow (u32, device; zero it first) is set when a region filled
 * (more than mean + 8 sigma + 64 keys in one coarse bucket: heavily duplicated content); the
 * grouping stays exact — that region's table workgroup regroups it from the whole d_keys
 * array on the device — so the flag only reports the slower path.  Batches the fused chain does not
 * take (n not a multiple of sd_cas_batch_quantum, n > 1,441,792, or a non-AUTO/HASH group
 * method) run the two calls in sequence, d_overflow untouched.  The Object count of an async
 * call: sd_cas_copy_objects_dev. */
int sd_cas_hash_group_sampled_dev(sd_cas_ctx* ctx, const void* d_content, uint64_t stride,
                                  const uint64_t* d_sizes, size_t n, uint64_t* d_keys,
                                  uint32_t* d_rep, uint32_t* d_overflow, uint64_t* out_objects,
                                  void* stream);
/* The same chain in its two halves, for callers that pipeline batches: hash_regions = K1 +
 * the partition into one of the context's two region sets (n a multiple of the quantum, <=
 * 1,441,792, default group method: else SD_CAS_EINVAL), async; group_regions = the bucket
 * tables over the regions of the LAST hash_regions batch (same n and d_rep: hash_regions
 * prefilled it), on any stream (the library orders it after that batch's K1), async unless
 * out_objects != NULL; d_keys of that batch must stay unchanged until its tables completed
 * (an overflowed region is regrouped from them).  A batch that is hashed but never grouped is
 * simply dropped by the next hash_regions into its set.  The sets alternate, so batch i's
 * tables may run on a side stream while batch i+1 hashes; a set is refilled only after its
 * previous K1 and tables finished (the library orders that itself).  d_overflow as above. */
int sd_cas_hash_regions_sampled_dev(sd_cas_ctx* ctx, const void* d_content, uint64_t stride,
                                    const uint64_t* d_sizes, size_t n, uint64_t* d_keys,
                                    uint32_t* d_rep, uint32_t* d_overflow, void* stream);
int sd_cas_group_regions_dev(sd_cas_ctx* ctx, size_t n, uint32_t* d_rep, uint64_t* out_objects,
                             void* stream);
/* Generalised grouping (the receive side of the multi-GPU exchange):
 * d_out[i] = min{ vals[j] : key[j] == key[i] } (vals NULL = identity, i.e. sd_cas_group_dev);
 * *out_objects = distinct keys (blocks when non-NULL).  n < 2^32 (above
 * SD_CAS_HASH_GROUP_MAX_KEYS: two stable LSD sorts, by value then by key). */
int sd_cas_group_min_dev(sd_cas_ctx* ctx, const uint64_t* d_keys, const uint32_t* d_vals, size_t n,
                         uint32_t* d_out, uint64_t* out_objects, void* stream);
/* Key-range partition for the exchange: part(k) = floor(k * parts / 2^64) (BLAKE3 keys are
 * uniform).  d_keys_out / d_pos_out = keys and their input positions, part-contiguous in
 * part order (order inside a part unspecified); d_counts[p] (u64, device) = part sizes.
 * parts <= 16384. */
int sd_cas_partition_dev(sd_cas_ctx* ctx, const uint64_t* d_keys, size_t n, uint32_t parts,
                         uint64_t* d_keys_out, uint32_t* d_pos_out, uint64_t* d_counts,
                         void* stream);
/* Row packing of the per-process RCCL key-range exchange (one process per GPU,
 * spacedrive_amd/shard.py): d_rows[3j..3j+2] = (key lo32, key hi32,
 * u32(file0 + d_pos[j])) for the partition's output; split turns received rows back into
 * keys + u32 vals; unpack scatters the mirrored u32 reps to local file order,
 * d_rep[d_pos[j]] = d_back[j] (u64).  file0 + n must fit in u32. */
int sd_cas_exchange_pack_dev(sd_cas_ctx* ctx, const uint64_t* d_keys, const uint32_t* d_pos,
                             size_t n, uint64_t file0, uint32_t* d_rows, void* stream);
int sd_cas_exchange_split_dev(sd_cas_ctx* ctx, const uint32_t* d_rows, size_t m,
                              uint64_t* d_keys, uint32_t* d_vals, void* stream);
int sd_cas_exchange_unpack_dev(sd_cas_ctx* ctx, const uint32_t* d_back, const uint32_t* d_pos,
                               size_t n, uint64_t* d_rep, void* stream);
/* Fixed-capacity form of the exchange rows (no host read of the part sizes): G blocks of
 * `cap` rows (d_rows, 3 u32 each) and G spill blocks of `spill` rows (d_spill_rows) are
 * always written — part p's first cap rows, its next spill rows, and in every unused slot a
 * sentinel row whose key is the first key of range p+1 (outside receiver p's range) and
 * whose value is 0xFFFFFFFF.  d_counts = the partition's part sizes (device).  A part
 * larger than cap + spill sets *d_overflow (u32, device; zero it first): the caller then
 * falls back to the exact exchange.  G <= 1024. */
int sd_cas_exchange_pack_fixed_dev(sd_cas_ctx* ctx, const uint64_t* d_keys, const uint32_t* d_pos,
                                   const uint64_t* d_counts, uint32_t G, uint64_t cap,
                                   uint64_t spill, uint64_t file0, uint32_t* d_rows,
                                   uint32_t* d_spill_rows, uint32_t* d_overflow, void* stream);
/* received rows -> keys + vals.  `sentinel` = this receiver's sentinel (the first key of
 * range rank+1); received row j carrying it gets the distinct key sentinel + j (outside the
 * receiver's range, so the padding spreads over the grouping's buckets instead of forming one
 * hot key) and *d_sentinel_rows (device u64; zero it first) += the number of such rows: each
 * is one extra Object of the grouping, to be subtracted from its count. */
int sd_cas_exchange_split_fixed_dev(sd_cas_ctx* ctx, const uint32_t* d_rows, size_t m,
                                    uint64_t sentinel, uint64_t* d_keys, uint32_t* d_vals,
                                    uint64_t* d_sentinel_rows, void* stream);
/* mirror of pack_fixed: d_rep[d_pos[o_p + t]] = (main or spill block) rep for t < count_p. */
int sd_cas_exchange_unpack_fixed_dev(sd_cas_ctx* ctx, const uint32_t* d_back,
                                     const uint32_t* d_spill_back, const uint32_t* d_pos,
                                     const uint64_t* d_counts, uint32_t G, uint64_t cap,
                                     uint64_t spill, uint64_t* d_rep, void* stream);
/* Enqueue a copy of the Object count of this context's last grouping call (sd_cas_group*_dev)
 * to device memory — for callers that keep the count on the device (no host sync). */
int sd_cas_copy_objects_dev(sd_cas_ctx* ctx, uint64_t* d_dst, void* stream);
/* Same on already-sorted pairs (keys ascending, vals = file idx, stable). */
int sd_cas_group_sorted_dev(sd_cas_ctx* ctx, const uint64_t* d_sorted_keys,
                            const uint32_t* d_sorted_vals, size_t n, uint32_t* d_rep,
                            uint64_t* out_objects, void* stream);
/* Reference chunk replay (identifier_job_step over CHUNK_SIZE rows, HashMap order :=
 * ascending idx): d_rep_chunked[i] = i if file i creates a new Object, else the file
 * whose Object it links to; *out_created / *out_linked = the summed per-step
 * (total_created, total_linked) of mod.rs:349.  Blocking. */
int sd_cas_group_chunked_dev(sd_cas_ctx* ctx, const uint32_t* d_rep, size_t n, uint32_t chunk,
                             uint32_t* d_rep_chunked, uint64_t* out_created,
                             uint64_t* out_linked, void* stream);
/* ---- Object-link emission of a file-identifier job ------------------
 * The decisions of file_identifier_job.rs:180-236 (the step loop) and identifier_job_step
 * (mod.rs:98-350) over n orphan file_path rows in ascending id order on a fresh library
 * (a library that already holds Objects: sd_cas_identifier_links_seeded below),
 * `chunk` rows per step (CHUNK_SIZE = 100, mod.rs:34), with the reference's cursor: step k
 * queries the orphan rows with `id >= cursor` (file_identifier_job.rs:268, 307-315) and
 * the next cursor is the chunk's LAST row (mod.rs:401-405), so a last row that stays
 * orphan (an error, or an empty file: no cas_id) is queried again by the next step; the
 * job runs at most ceil(n / chunk) steps (file_identifier_job.rs:146) and ends early when
 * a query comes back empty.
 *   d_keys[i]  cas key of row i (read for hashed rows only)
 *   rows       the file_paths the job's orphan query returns: object_id or cas_id NULL,
 *              not a directory, and indexed size_in_bytes != 0 (orphan_path_filters,
 *              file_identifier_job.rs:251-277) — a file indexed empty is never a row.
 *              These calls model rows with object_id NULL; rows that already hold an
 *              Object (object_id set, cas_id NULL) need sd_cas_identifier_links_ex below.
 *              A stale cas_id on a row without an Object changes nothing (it is rewritten
 *              before find_many and connects no Object)
 *   d_state[i] SD_CAS_ROW_* (u8; NULL = every row hashed): HASHED = cas_id computed,
 *              NO_CAS = fs::metadata length 0 at identification time (a file emptied
 *              after indexing: no cas_id, mod.rs:78-86), ERROR = FileMetadata::new failed
 *              (the row is dropped from its step, mod.rs:125-141)
 * Outputs (device, n entries each):
 *   d_step[i]   the (last) step that processed row i, SD_CAS_NO_STEP if none;
 *   d_object[i] the row whose new Object row i is connected to: i when row i created one
 *               (create_many, mod.rs:246-347), the key's first row when it linked to an
 *               existing Object (mod.rs:202-238; find() = the lowest Object id), and
 *               SD_CAS_NO_OBJECT when dropped or not reached;
 *   d_action[i] SD_CAS_LINK_*.
 * h_step_counts (host, 2 x max_steps u64): per step (total_created, total_linked) as
 * identifier_job_step returns them (mod.rs:349); an empty row queried again counts one
 * creation in every step that processed it.  *out_steps = steps executed.  Ties inside a
 * step follow HashMap order := ascending row.  Blocking; n < 2^32. */
#define SD_CAS_ROW_HASHED 0
#define SD_CAS_ROW_NO_CAS 1
#define SD_CAS_ROW_ERROR 2
#define SD_CAS_LINK_CREATED 0
#define SD_CAS_LINK_LINKED 1
#define SD_CAS_LINK_DROPPED 2
#define SD_CAS_LINK_NOT_REACHED 3
#define SD_CAS_LINK_EXISTING 4
#define SD_CAS_NO_STEP 0xFFFFFFFFu
#define SD_CAS_NO_OBJECT 0xFFFFFFFFu
size_t sd_cas_identifier_max_steps(size_t n, uint32_t chunk);
int sd_cas_identifier_links_dev(sd_cas_ctx* ctx, const uint64_t* d_keys, const uint8_t* d_state,
                                size_t n, uint32_t chunk, uint32_t* d_step, uint32_t* d_object,
                                uint8_t* d_action, uint64_t* h_step_counts, size_t max_steps,
                                uint64_t* out_steps, void* stream);
/* Same with every array in host memory (the DB layer's side of the boundary: keys and
 * per-file status come from sd_cas_generate_cas_ids_from_paths, the decisions go into the
 * create_many / link batches).  h_state NULL = every row hashed.  Blocking. */
int sd_cas_identifier_links(sd_cas_ctx* ctx, const uint64_t* h_keys, const uint8_t* h_state,
                            size_t n, uint32_t chunk, uint32_t* h_step, uint32_t* h_object,
                            uint8_t* h_action, uint64_t* h_step_counts, size_t max_steps,
                            uint64_t* out_steps);
/* The same job on a library that already holds Objects (an incremental job, or a second
 * location of the same library): every step's find_many (mod.rs:180-198) returns the
 * Objects already connected to ANY file_path with one of the step's cas_ids — there is no
 * location filter — so a row whose key such an Object carries links to it (mod.rs:202-238,
 * find() = the first Object in id order) and its key never creates (mod.rs:246-253).
 * seed_keys[j] / seed_objects[j] (n_seed pairs, any order, repeats allowed) = (cas key, id)
 * of each Object that exists before the job and is connected to a file_path with that
 * cas_id, as the DB returns them; ids < 2^31, ascending in the DB's row order.  Such a row
 * gets action SD_CAS_LINK_EXISTING, object = the SMALLEST id seeded for its key, and counts
 * as linked in its step.  n_seed = 0 is the fresh-library call above; seeded calls need
 * n < 2^31. */
int sd_cas_identifier_links_seeded_dev(sd_cas_ctx* ctx, const uint64_t* d_keys, const uint8_t* d_state,
                                       size_t n, uint32_t chunk, const uint64_t* d_seed_keys,
                                       const uint32_t* d_seed_objects, size_t n_seed, uint32_t* d_step,
                                       uint32_t* d_object, uint8_t* d_action, uint64_t* h_step_counts,
                                       size_t max_steps, uint64_t* out_steps, void* stream);
int sd_cas_identifier_links_seeded(sd_cas_ctx* ctx, const uint64_t* h_keys, const uint8_t* h_state,
                                   size_t n, uint32_t chunk, const uint64_t* h_seed_keys,
                                   const uint32_t* h_seed_objects, size_t n_seed, uint32_t* h_step,
                                   uint32_t* h_object, uint8_t* h_action, uint64_t* h_step_counts,
                                   size_t max_steps, uint64_t* out_steps);
/* The same job with rows that ALREADY OWN an Object: the orphan query is `object_id IS NULL OR
 * cas_id IS NULL` (file_identifier_job.rs:258-261), so a file_path with an Object but no
 * cas_id is a row — the watcher's sequence for a file created empty (it gets an Object with
 * no cas_id, watcher/utils.rs:236-293) and then written (the update keeps the old NULL
 * cas_id, :473-490).  pre_objects[i] = the Object id row i's file_path holds (< 2^31, ids
 * ascending in the DB's row order like the seeds) or SD_CAS_NO_OBJECT; NULL = none.
 * Semantics (mod.rs:157-253): the step that processes a HASHED row writes its cas_id X
 * first, so that step's find_many also returns the row's Object under X: every row of the
 * step with key X links to the smallest Object id carrying X (seeds, pre-existing Objects of
 * X rows processed in this or an earlier step, and — only when no pre-job Object carries X —
 * the Object created for X's first row) and X never creates.  A pre-existing Object can
 * therefore take over a key that an earlier step created an Object for: rows of later
 * steps link to it (SD_CAS_LINK_EXISTING).  The row itself is re-linked (counted as linked),
 * also to a smaller Object than its own.  A NO_CAS row with an Object still creates a new
 * one (mod.rs:248-253) and an ERROR row keeps its Object, stays orphan and is DROPPED; for
 * both d_object says what the job did (i / SD_CAS_NO_OBJECT), not the untouched column.
 * Ids >= 2^31 other than SD_CAS_NO_OBJECT, in seeds or pre_objects, fail with SD_CAS_EINVAL
 * (the device call checks them on the device).  pre_objects != NULL costs one pass over the
 * rows' states and Objects, then work on the EVENTS only — the hashed rows holding an Object:
 * a stable sort of their keys, two segmented-min scans, and per hashed row a lookup of its
 * key (a 1 MiB key bitmap, then a binary search).  n < 2^31. */
int sd_cas_identifier_links_ex_dev(sd_cas_ctx* ctx, const uint64_t* d_keys, const uint8_t* d_state,
                                   size_t n, uint32_t chunk, const uint64_t* d_seed_keys,
                                   const uint32_t* d_seed_objects, size_t n_seed,
                                   const uint32_t* d_pre_objects, uint32_t* d_step,
                                   uint32_t* d_object, uint8_t* d_action, uint64_t* h_step_counts,
                                   size_t max_steps, uint64_t* out_steps, void* stream);
int sd_cas_identifier_links_ex(sd_cas_ctx* ctx, const uint64_t* h_keys, const uint8_t* h_state,
                               size_t n, uint32_t chunk, const uint64_t* h_seed_keys,
                               const uint32_t* h_seed_objects, size_t n_seed,
                               const uint32_t* h_pre_objects, uint32_t* h_step, uint32_t* h_object,
                               uint8_t* h_action, uint64_t* h_step_counts, size_t max_steps,
                               uint64_t* out_steps);

/* Stable LSD radix sort of (u64 key, u32 val) on bits [begin_bit, end_bit).
 * d_vals_in == NULL sorts the identity 0..n-1. */
int sd_cas_sort_pairs_dev(sd_cas_ctx* ctx, const uint64_t* d_keys_in, const uint32_t* d_vals_in,
                          size_t n, uint64_t* d_keys_out, uint32_t* d_vals_out, int begin_bit,
                          int end_bit, void* stream);

/* ---- file_checksum (validation/hash.rs:11-25) ------------------------------------------
 * Full BLAKE3 digest (32 B) of a device buffer (16-B aligned, readable to the 16-B round-up
 * of len).  Blocking. */
int sd_cas_checksum_dev(sd_cas_ctx* ctx, const void* d_data, uint64_t len, uint8_t out[32],
                        void* stream);
/* file_checksum(path): the bytes hash.rs:15-21 hashes — its loop issues 1 MiB read()s and
 * stops after the FIRST read shorter than 1 MiB, which is EOF on a local regular file but
 * not on a procfs seq_file (about one page per read), a FIFO or a FUSE/network mount.
 * Regular files are read in parallel (pread pieces) and streamed through pinned staging in
 * 64 MiB segments, one BLAKE3 subtree per segment on the GPU; a regular file whose reads
 * come back short before its end (or that ends before st_size), and every non-regular
 * file, is read as hash.rs reads it: sequential 1 MiB read()s from the start up to and
 * including the first short one.  out_hex = 64 lowercase hex + NUL.
 * Returns SD_CAS_EIO with *err_no set on an I/O error. */
int sd_cas_file_checksum(sd_cas_ctx* ctx, const char* path, char out_hex[65], int* err_no);
/* The validator job over many files (validator_job.rs:107-172 runs one file_checksum per
 * step): n device buffers hashed by one launch chain — buffer i = d_arena + d_offs[i]
 * (16-B aligned), d_lens[i] bytes (<= 64 GiB), readable to the 16-B round-up; every buffer
 * ends within arena_bytes of d_arena (sizes the workspace: one 32-B CV per 1 MiB subtree).
 * d_out[32 i .. 32 i + 32) = the digest of buffer i (device).  n <= 2^24.  Blocking;
 * SD_CAS_EINVAL when a buffer breaks those bounds (it is then not read). */
int sd_cas_checksums_dev(sd_cas_ctx* ctx, const void* d_arena, uint64_t arena_bytes,
                         const uint64_t* d_offs, const uint64_t* d_lens, size_t n, uint8_t* d_out,
                         void* stream);
/* file_checksum over n paths, each with sd_cas_file_checksum's result: regular files are
 * read by the gather pool into pinned windows that are hashed with the batch chain above while
 * the next window is read; a file larger than half a window, one that grew past its slot, a
 * non-regular file, and one whose reads came back short before its end or that ended before
 * st_size (hash.rs:15-21 would stop at its first short read) go through
 * sd_cas_file_checksum.  out_hex[65 i ..] = 64 hex + NUL ("" on error);
 * status[i] = 0 or -errno (open/stat/read failure: validator_job.rs:149-151 fails that
 * step with FileIOError).  Returns SD_CAS_OK unless the batch itself failed.  Blocking. */
int sd_cas_file_checksums(sd_cas_ctx* ctx, const char* const* paths, size_t n, char* out_hex,
                          int32_t* status);

/* ---- multi-device, single process -------------------------------------
 * One context per shard; shard i lives on devices[i] (a device may host several shards).
 * Grouping pulls each shard's key range from every other shard with peer copies over
 * xGMI (hipMemcpyPeerAsync, event-ordered across devices), then groups locally; the
 * multi-process form of the same exchange uses RCCL all-to-all (spacedrive_amd/shard.py). */
typedef struct sd_cas_multi sd_cas_multi;
/* Fails with SD_CAS_ENODEV when a device is not a gfx950 or when peer access between two
 * distinct devices cannot be enabled (sd_cas_multi_last_error(NULL) says which). */
int sd_cas_multi_create(const int* devices, int ndev, sd_cas_multi** out);
void sd_cas_multi_destroy(sd_cas_multi* m);
int sd_cas_multi_count(const sd_cas_multi* m);
sd_cas_ctx* sd_cas_multi_ctx(sd_cas_multi* m, int i);
const char* sd_cas_multi_last_error(const sd_cas_multi* m);
/* Canonical grouping across shards: shard i holds n[i] keys (device pointer on its
 * device) for files file0[i] .. file0[i]+n[i]-1 (file0 ascending, ranges disjoint);
 * d_rep[i][k] (u64, device) = global idx of the file owning key k's Object;
 * *out_objects = total Objects.  Blocking. */
int sd_cas_multi_group(sd_cas_multi* m, const uint64_t* const* d_keys, const size_t* n,
                       const uint64_t* file0, uint64_t* const* d_rep, uint64_t* out_objects);
/* End to end from host memory: n sampled contents (57,344 B at h_content + i*stride) are
 * split into contiguous shards, streamed to their devices (H2D overlapped with K1, all
 * devices in flight), hashed and grouped.  h_keys[i] = cas key, h_rep[i] (optional) =
 * global idx of the file owning file i's Object.  Blocking. */
int sd_cas_multi_hash_group_sampled_host(sd_cas_multi* m, const void* h_content, uint64_t stride,
                                         const uint64_t* h_sizes, size_t n, uint64_t* h_keys,
                                         uint64_t* h_rep, uint64_t* out_objects);

/* ---- synthetic inputs (benchmarks / tests; same generator as oracle/cas_ref.c) ------- */
int sd_cas_synth_sampled_dev(sd_cas_ctx* ctx, uint64_t seed, uint64_t file0, size_t n,
                             uint32_t dup_permille, void* d_content, uint64_t stride,
                             uint64_t* d_sizes, void* stream);
/* whole-file path: fills d_sizes/d_lens, d_offs (128-B aligned packing) and the arena;
 * *out_arena_bytes = bytes used.  Pass d_arena == NULL to only size it (blocking). */
int sd_cas_synth_small_dev(sd_cas_ctx* ctx, uint64_t seed, uint64_t file0, size_t n,
                           uint32_t dup_permille, uint64_t* d_sizes, uint32_t* d_lens,
                           uint64_t* d_offs, void* d_arena, uint64_t* out_arena_bytes,
                           void* stream);
/* whole-file content only, at caller-chosen offsets (e.g. another alignment than the
 * 128-B packing above): file i's lens[i] bytes at d_arena + d_offs[i] (16-B aligned;
 * the quad holding the tail is written whole). */
int sd_cas_synth_small_content_dev(sd_cas_ctx* ctx, uint64_t seed, uint64_t file0, size_t n,
                                   uint32_t dup_permille, const uint64_t* d_offs,
                                   const uint32_t* d_lens, void* d_arena, void* stream);
/* bytes [byte_off, byte_off + len) of synthetic file `file`'s content stream (the
 * validator's multi-GiB files; byte_off and d_out 8-B aligned, d_out writable to the 8-B
 * round-up of len) */
int sd_cas_synth_stream_dev(sd_cas_ctx* ctx, uint64_t seed, uint64_t file, uint64_t byte_off,
                            uint64_t len, void* d_out, void* stream);
int sd_cas_synth_roots_dev(sd_cas_ctx* ctx, uint64_t seed, uint64_t file0, size_t n,
                           uint32_t dup_permille, uint64_t* d_roots, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* SD_HIP_CAS_H */
