// sd_hip_cas.cpp — the C ABI (include/sd_hip_cas.h) over the gfx950 kernels.
//
// Host runtime for the batched drop-in of generate_cas_id (core/src/object/cas.rs:23-62),
// its batch caller identifier_job_step (core/src/object/file_identifier/mod.rs:98-350)
// and file_checksum (core/src/object/validation/hash.rs:11-25):
//   - a context per (thread, device): compute stream + copy (side) stream, a growable
//     device workspace and pinned staging, last-error string;
//   - host batches are gathered into pinned staging (pread at the cas.rs:27-58 offsets
//     for the path variant), copied with hipMemcpyAsync on the side stream, and hashed
//     on the compute stream after an event hand-off;
//   - no CPU hashing anywhere: every digest comes from the HIP kernels.
#include <errno.h>
#include <fcntl.h>
#include <hip/hip_runtime.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <memory>
#include <string>
#include <thread>
#include <vector>

#include "sd_checksum.h"
#include "sd_group.h"
#include "sd_kernels.h"
#include "sd_links.h"
#include "sd_mix.h"
#include "sd_synth.h"

using namespace sdcas;

#include "sd_debug.h"
#if SD_DBG
namespace sdcas {
uint32_t sd_dbg_violations_group_hash();
uint32_t sd_dbg_violations_group();
uint32_t sd_dbg_violations_checksum();
}  // namespace sdcas
// debug library only (libsd_hip_cas_debug.so, not in the ABI header): invariant violations
// counted by the device checks of sd_debug.h since the library was loaded
extern "C" uint64_t sd_cas_debug_violations(void) {
  return (uint64_t)sd_dbg_violations_group_hash() + sd_dbg_violations_group() +
         sd_dbg_violations_checksum();
}
#endif

#include "ctx_internal.h"

// short local names for the shared helpers
#define fail sd_fail
#define pick sd_pick
#define ensure sd_ensure
#define ensure_pinned sd_ensure_pinned

extern "C" {

int sd_cas_abi_version(void) { return SD_CAS_ABI_VERSION; }

// why the calling thread's last sd_cas_ctx_create failed: sd_cas_last_error(NULL)
static thread_local std::string g_ctx_create_err;

int sd_cas_ctx_create(int device, sd_cas_ctx** out) {
  if (!out) return SD_CAS_EINVAL;
  *out = nullptr;
  g_ctx_create_err.clear();
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) {
    (void)hipGetLastError();
    g_ctx_create_err = "no HIP device " + std::to_string(device) + " (" + std::to_string(ndev) +
                       " visible)";
    return SD_CAS_ENODEV;
  }
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) != hipSuccess) {
    g_ctx_create_err = "hipGetDeviceProperties(" + std::to_string(device) + ") failed";
    return SD_CAS_ENODEV;
  }
  if (strncmp(prop.gcnArchName, "gfx950", 6) != 0) {  // gfx950 only
    g_ctx_create_err = std::string("device ") + std::to_string(device) + " is " + prop.gcnArchName +
                       ", not gfx950 (MI355X)";
    return SD_CAS_ENODEV;
  }
  sd_cas_ctx* c = new sd_cas_ctx();
  c->device = device;
  if (hipSetDevice(device) != hipSuccess ||
      hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
      hipStreamCreateWithFlags(&c->copy, hipStreamNonBlocking) != hipSuccess ||
      hipStreamCreateWithFlags(&c->copy2, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreateWithFlags(&c->copy2_done, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&c->h2d_done, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&c->packed_h2d, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&c->packed_done, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&c->ws_ev, hipEventDisableTiming) != hipSuccess ||
      hipMalloc((void**)&c->d_scalar, 64) != hipSuccess ||
      hipMalloc((void**)&c->gtotals, GROUP_TOTALS_WORDS * 4) != hipSuccess ||
      hipMemset(c->gtotals, 0, GROUP_TOTALS_WORDS * 4) != hipSuccess ||
      hipMalloc((void**)&c->gcursor, 2 * REGION_SET_WORDS * 4) != hipSuccess ||
      hipMemset(c->gcursor, 0, 2 * REGION_SET_WORDS * 4) != hipSuccess ||
      hipEventCreateWithFlags(&c->region_done[0], hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&c->region_done[1], hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&c->region_hashed[0], hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&c->region_hashed[1], hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&c->gather_done[0], hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&c->gather_done[1], hipEventDisableTiming) != hipSuccess) {
    sd_cas_ctx_destroy(c);
    g_ctx_create_err = "stream/event/scratch creation failed on device " + std::to_string(device);
    return SD_CAS_EHIP;
  }
  c->quantum = (size_t)prop.multiProcessorCount * 4 * 64;
  {
    const char* t = getenv("SD_CAS_TRACE");
    c->trace = t && *t && strcmp(t, "0") != 0;
  }
  sd_cas_set_latency_threshold(c, SD_CAS_THRESHOLD_DEFAULT, SD_CAS_THRESHOLD_DEFAULT);
  sd_cas_set_chunkpar_split(c, SD_CAS_THRESHOLD_DEFAULT, SD_CAS_THRESHOLD_DEFAULT);
  *out = c;
  return SD_CAS_OK;
}

// Defaults = the measured crossovers on MI355X (profiles/r01_k1l_seg_sweep.log,
// r02_latency_sweep.log): K1L (four files per wave) wins below ~0.75 of a batch quantum for
// sampled messages (49,152 files: 1.11 vs 1.15 ms; 65,536: 1.47 vs 1.19) and below ~2
// quanta for ragged whole files (98,304: 2.47 vs 2.80 ms; 131,072: 3.28 vs 3.24; 163,840:
// 4.08 vs 3.96 — round 2's K2 fast path moved this from ~3 quanta), where the lane-per-file
// K2 waits for the 101-chunk latency of its longest files.
void sd_cas_set_latency_threshold(sd_cas_ctx* c, size_t sampled_files, size_t packed_files) {
  if (!c) return;
  const size_t q = sd_cas_batch_quantum(c);
  c->latency_sampled = sampled_files == SD_CAS_THRESHOLD_DEFAULT ? q * 3 / 4 : sampled_files;
  c->latency_packed = packed_files == SD_CAS_THRESHOLD_DEFAULT ? q * 2 : packed_files;
}

// Defaults = the measured crossovers between the two K1L shapes (profiles/
// r01_k1l_seg_sweep.log): a wave per file while the batch cannot fill the chip's SIMDs,
// four files per wave once the lower wave-compression count per file wins.
void sd_cas_set_chunkpar_split(sd_cas_ctx* c, size_t sampled_files, size_t packed_files) {
  if (!c) return;
  // sampled: crossover between 2,048 (0.078 vs 0.116 ms) and 4,096 files (0.139 vs 0.120);
  // ragged whole files (visited by chunk count, so a wave's 4 files share a chunks-per-lane
  // class; the sort costs ~15 us): between 4,096 (0.216 vs 0.247) and 8,192 (0.364 vs 0.324)
  const size_t q = sd_cas_batch_quantum(c);
  c->seg16_sampled = sampled_files == SD_CAS_THRESHOLD_DEFAULT ? q * 3 / 64 : sampled_files;
  c->seg16_packed = packed_files == SD_CAS_THRESHOLD_DEFAULT ? q * 3 / 32 : packed_files;
}

void sd_cas_ctx_destroy(sd_cas_ctx* c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  (void)hipDeviceSynchronize();
  if (c->ws.p) (void)hipFree(c->ws.p);
  if (c->staging.p) (void)hipFree(c->staging.p);
  if (c->small.p) (void)hipFree(c->small.p);
  if (c->cvbuf.p) (void)hipFree(c->cvbuf.p);
  if (c->io.p) (void)hipFree(c->io.p);
  if (c->d_scalar) (void)hipFree(c->d_scalar);
  if (c->gtotals) (void)hipFree(c->gtotals);
  if (c->gcursor) (void)hipFree(c->gcursor);
  for (int k = 0; k < 2; k++) {
    if (c->regions[k].p) (void)hipFree(c->regions[k].p);
    if (c->region_done[k]) (void)hipEventDestroy(c->region_done[k]);
    if (c->region_hashed[k]) (void)hipEventDestroy(c->region_hashed[k]);
  }
  for (int b = 0; b < 2; b++)
    if (c->gather_done[b]) (void)hipEventDestroy(c->gather_done[b]);
  if (c->pinned) (void)hipHostFree(c->pinned);
  if (c->h2d_done) (void)hipEventDestroy(c->h2d_done);
  if (c->packed_h2d) (void)hipEventDestroy(c->packed_h2d);
  if (c->packed_done) (void)hipEventDestroy(c->packed_done);
  if (c->ws_ev) (void)hipEventDestroy(c->ws_ev);
  if (c->copy) (void)hipStreamDestroy(c->copy);
  if (c->copy2) (void)hipStreamDestroy(c->copy2);
  if (c->copy2_done) (void)hipEventDestroy(c->copy2_done);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
}

const char* sd_cas_last_error(const sd_cas_ctx* c) {
  return c ? c->err.c_str() : g_ctx_create_err.empty() ? "null context" : g_ctx_create_err.c_str();
}

void* sd_cas_ctx_stream(sd_cas_ctx* c) { return c ? (void*)c->stream : nullptr; }

size_t sd_cas_batch_quantum(const sd_cas_ctx* c) { return c ? c->quantum : 0; }

int sd_cas_set_group_method(sd_cas_ctx* c, int method, uint64_t bucket_target) {
  if (!c) return SD_CAS_EINVAL;
  if (method < SD_CAS_GROUP_AUTO || method > SD_CAS_GROUP_SORT || (bucket_target && bucket_target < 16))
    return fail(c, SD_CAS_EINVAL, "set_group_method: method %d, bucket_target %llu", method,
                (unsigned long long)bucket_target);
  c->group_method = method;
  c->group_target = bucket_target;
  return SD_CAS_OK;
}

int sd_cas_synchronize(sd_cas_ctx* c) {
  if (!c) return SD_CAS_EINVAL;
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  return SD_CAS_OK;
}

int sd_cas_alloc_pinned(sd_cas_ctx* c, size_t bytes, void** out) {
  if (!c || !out) return SD_CAS_EINVAL;
  if (hipHostMalloc(out, bytes ? bytes : 1, hipHostMallocDefault) != hipSuccess) {
    (void)hipGetLastError();
    return fail(c, SD_CAS_ENOMEM, "hipHostMalloc(%zu) failed", bytes);
  }
  return SD_CAS_OK;
}

int sd_cas_free_pinned(sd_cas_ctx* c, void* p) {
  if (!c) return SD_CAS_EINVAL;
  HIP_TRY(c, hipHostFree(p));
  return SD_CAS_OK;
}

void sd_cas_key_to_hex(uint64_t key, char out[17]) {
  static const char* hx = "0123456789abcdef";
  for (int i = 0; i < 16; i++) out[i] = hx[(key >> (60 - 4 * i)) & 15];
  out[16] = 0;
}

// ---- device-resident cas ----------------------------------------------------------

// Sampled batch dispatch.  Below the latency threshold: K1L.  Otherwise K1 over whole batch
// quanta (one file per lane fills every SIMD's wave slots exactly) and the remainder r:
// with K1 as well when r >= the threshold, else K1L after it — a partial K1 wave round
// costs a whole K1 latency however few files it holds (profiles/r01_k1l_seg_sweep.log:
// 98,304 files 2.34 ms on K1 alone vs 1.26 + 0.76 ms split).
static hipError_t dispatch_sampled(sd_cas_ctx* c, const uint8_t* content, uint64_t stride,
                                   const uint64_t* sizes, size_t n, uint64_t* keys,
                                   hipStream_t s) {
  if (n < c->latency_sampled)
    return hash_chunkpar(content, nullptr, stride, nullptr, SAMPLED_CONTENT_LEN, sizes, n, keys,
                         c->chunkpar_seg(n, true), s);
  const size_t q = c->quantum;
  const size_t r = n % q;
  const uint32_t cus = (uint32_t)(q / 256);
  if (n < q || r == 0 || r >= c->latency_sampled) return hash_sampled(content, stride, sizes, n, keys, s, cus);
  const size_t full = n - r;
  hipError_t e = hash_sampled(content, stride, sizes, full, keys, s, cus);
  if (e != hipSuccess) return e;
  return hash_chunkpar(content + full * stride, nullptr, stride, nullptr, SAMPLED_CONTENT_LEN,
                       sizes + full, r, keys + full, c->chunkpar_seg(r, true), s);
}

int sd_cas_hash_sampled_dev(sd_cas_ctx* c, const void* d_content, uint64_t stride,
                            const uint64_t* d_sizes, size_t n, uint64_t* d_keys, void* stream) {
  if (!c) return SD_CAS_EINVAL;
  if (n == 0) return SD_CAS_OK;
  if (!d_content || !d_sizes || !d_keys || stride < SAMPLED_CONTENT_LEN || (stride & 15) ||
      ((uintptr_t)d_content & 15))
    return fail(c, SD_CAS_EINVAL, "hash_sampled: bad content/stride (stride=%llu)",
                (unsigned long long)stride);
  HIP_TRY(c, dispatch_sampled(c, (const uint8_t*)d_content, stride, d_sizes, n, d_keys,
                              pick(c, stream)));
  return SD_CAS_OK;
}

int sd_cas_hash_packed_dev(sd_cas_ctx* c, const void* d_arena, const uint64_t* d_offs,
                           const uint32_t* d_lens, const uint64_t* d_sizes, size_t n,
                           uint64_t* d_keys, void* stream) {
  if (!c) return SD_CAS_EINVAL;
  if (n == 0) return SD_CAS_OK;
  if (!d_arena || !d_offs || !d_lens || !d_sizes || !d_keys || ((uintptr_t)d_arena & 15) ||
      n >= (1ull << 32))
    return fail(c, SD_CAS_EINVAL, "hash_packed: bad arguments");
  hipStream_t s = pick(c, stream);
  const bool k1l = n < c->latency_packed;
  if (k1l && c->chunkpar_seg(n, false) == 64) {  // small batch: a wave per file, no sort
    HIP_TRY(c, hash_chunkpar((const uint8_t*)d_arena, d_offs, 0, d_lens, 0, d_sizes, n, d_keys,
                             64, s));
    return SD_CAS_OK;
  }
  // K2, and K1L with 4 files per wave: visit the files by descending chunk count (one
  // stable radix pass) so the lanes of a wave (K2) / the files of a wave (K1L) match.
  // workspace: length keys | sorted keys | order | sort workspace
  const size_t kb = up256(n * 8), ob = up256(n * 4);
  int rc = ensure(c, c->ws, 2 * kb + ob + sort_workspace_bytes(n));
  if (rc) return rc;
  char* p = (char*)c->ws.p;
  uint64_t* lkeys = (uint64_t*)p;
  uint64_t* skeys = (uint64_t*)(p + kb);
  uint32_t* order = (uint32_t*)(p + 2 * kb);
  void* sws = p + 2 * kb + ob;
  HIP_TRY(c, sd_ws_acquire(c, s));
  HIP_TRY(c, length_keys(d_lens, n, lkeys, s));
  HIP_TRY(c, radix_sort_pairs(lkeys, nullptr, skeys, order, n, 0, length_key_bits(n), sws, s));
  if (k1l)
    HIP_TRY(c, hash_chunkpar((const uint8_t*)d_arena, d_offs, 0, d_lens, 0, d_sizes, n, d_keys,
                             16, s, order));
  else
    HIP_TRY(c, hash_packed((const uint8_t*)d_arena, d_offs, d_lens, d_sizes, order, n, d_keys, s));
  HIP_TRY(c, sd_ws_release(c, s));
  return SD_CAS_OK;
}

// ---- grouping -----------------------------------------------------------------------

int sd_cas_sort_pairs_dev(sd_cas_ctx* c, const uint64_t* d_keys_in, const uint32_t* d_vals_in,
                          size_t n, uint64_t* d_keys_out, uint32_t* d_vals_out, int begin_bit,
                          int end_bit, void* stream) {
  if (!c) return SD_CAS_EINVAL;
  if (n == 0) return SD_CAS_OK;
  if (!d_keys_in || !d_keys_out || !d_vals_out || n >= (1ull << 32) || begin_bit < 0 ||
      end_bit > 64 || begin_bit >= end_bit)
    return fail(c, SD_CAS_EINVAL, "sort_pairs: bad arguments");
  int rc = ensure(c, c->ws, sort_workspace_bytes(n));
  if (rc) return rc;
  hipStream_t s = pick(c, stream);
  HIP_TRY(c, sd_ws_acquire(c, s));
  HIP_TRY(c, radix_sort_pairs(d_keys_in, d_vals_in, d_keys_out, d_vals_out, n, begin_bit, end_bit,
                              c->ws.p, s));
  HIP_TRY(c, sd_ws_release(c, s));
  return SD_CAS_OK;
}

int sd_cas_group_dev(sd_cas_ctx* c, const uint64_t* d_keys, size_t n, uint32_t* d_rep,
                     uint64_t* out_objects, void* stream) {
  if (!c) return SD_CAS_EINVAL;
  if (n >= (1ull << 32) || (n && (!d_keys || !d_rep)))
    return fail(c, SD_CAS_EINVAL, "group: bad arguments");
  if (c->group_method == SD_CAS_GROUP_HASH && !hash_group_supported(n))
    return fail(c, SD_CAS_EINVAL, "group: %zu keys exceed the hash grouping's range", n);
  hipStream_t s = pick(c, stream);
  if (c->use_hash_group(n)) {  // K4h/K5h: bucket partition + LDS hash min (no full sort)
    int rc = ensure(c, c->ws, hash_group_workspace_bytes(n, c->group_target));
    if (rc) return rc;
    HIP_TRY(c, sd_ws_acquire(c, s));
    HIP_TRY(c, hash_group_min(d_keys, nullptr, n, d_rep, c->d_scalar, c->ws.p, c->gtotals, s,
                              c->group_target));
  } else {  // beyond the hash grouping's range: LSD radix sort + run heads (K4 + K5)
    int rc = ensure(c, c->ws, group_workspace_bytes(n));
    if (rc) return rc;
    HIP_TRY(c, sd_ws_acquire(c, s));
    HIP_TRY(c, group_keys(d_keys, n, d_rep, c->d_scalar, c->ws.p, s));
  }
  HIP_TRY(c, sd_ws_release(c, s));
  c->region_obj_set = -1;
  if (out_objects) {
    HIP_TRY(c, hipMemcpyAsync(out_objects, c->d_scalar, 8, hipMemcpyDeviceToHost, s));
    HIP_TRY(c, hipStreamSynchronize(s));
  }
  return SD_CAS_OK;
}

// ---- the fused hash + group chain -------------------------------------------------
static bool fused_eligible(const sd_cas_ctx* c, size_t n) {
  return n && n % c->quantum == 0 && region_group_supported(n) &&
         (c->group_method == SD_CAS_GROUP_AUTO || c->group_method == SD_CAS_GROUP_HASH) &&
         c->group_target == 0;
}

// region set k's buffer: rkeys | rfile | gkeys | gvals | spill keys | spill files
// (region_group_layout) | objects u64 | overflow carve cursor u64
static uint64_t* region_objects(sd_cas_ctx* c, int k) {
  return (uint64_t*)((char*)c->regions[k].p + region_group_workspace_bytes(c->region_n[k]));
}

int sd_cas_hash_regions_sampled_dev(sd_cas_ctx* c, const void* d_content, uint64_t stride,
                                    const uint64_t* d_sizes, size_t n, uint64_t* d_keys,
                                    uint32_t* d_rep, uint32_t* d_overflow, void* stream) {
  if (!c) return SD_CAS_EINVAL;
  if (!fused_eligible(c, n))
    return fail(c, SD_CAS_EINVAL,
                "hash_regions: %zu files (a multiple of %zu up to 1,441,792, default group method)",
                n, c->quantum);
  if (!d_content || !d_sizes || !d_keys || !d_rep || !d_overflow || stride < SAMPLED_CONTENT_LEN ||
      (stride & 15) || ((uintptr_t)d_content & 15))
    return fail(c, SD_CAS_EINVAL, "hash_regions: bad arguments (stride=%llu)",
                (unsigned long long)stride);
  HIP_TRY(c, hipSetDevice(c->device));
  hipStream_t s = pick(c, stream);
  const int k = (c->region_cur + 1) & 1;
  // set k was last grouped two batches ago: its tables must be done before it is refilled;
  // a batch hashed into it but never grouped: its K1G (on whatever stream) must be done
  if (c->region_pending[k]) HIP_TRY(c, hipStreamWaitEvent(s, c->region_done[k], 0));
  if (!c->region_grouped[k]) {
    HIP_TRY(c, hipStreamWaitEvent(s, c->region_hashed[k], 0));
    // its cursors and spill count were left counted: clear them
    HIP_TRY(c, hipMemsetAsync(c->gcursor + REGION_SET_WORDS * k, 0, REGION_SET_WORDS * 4, s));
  }
  if (c->region_obj_set == k) {
    // set k holds the Object count of the context's last grouping, which this refill's K1G
    // zeroes: keep it in d_scalar for sd_cas_copy_objects_dev
    HIP_TRY(c, sd_ws_acquire(c, s));
    HIP_TRY(c, hipMemcpyAsync(c->d_scalar, region_objects(c, k), 8, hipMemcpyDeviceToDevice, s));
    HIP_TRY(c, sd_ws_release(c, s));
    c->region_obj_set = -1;
  }
  c->region_n[k] = n;  // sizes the layout (ensure below grows the set if needed)
  int rc = ensure(c, c->regions[k], region_group_workspace_bytes(n) + 256);
  if (rc) return rc;
  uint64_t *rkeys, *gkeys, *skeys;
  uint32_t *rfile, *gvals, *sfile;
  region_group_layout(c->regions[k].p, n, &rkeys, &rfile, &gkeys, &gvals, &skeys, &sfile);
  uint32_t* cur = c->gcursor + REGION_SET_WORDS * k;
  hipError_t e = hash_sampled_regions((const uint8_t*)d_content, stride, d_sizes, n, d_keys, d_rep,
                                      rkeys, rfile, cur, region_capacity(n), skeys, sfile, d_overflow,
                                      region_objects(c, k), s, (uint32_t)(c->quantum / 256));
  if (e != hipSuccess) {
    (void)hipMemsetAsync(cur, 0, REGION_SET_WORDS * 4, s);  // restore the cursors' invariant
    return fail(c, SD_CAS_EHIP, "hash_regions: %s", hipGetErrorString(e));
  }
  HIP_TRY(c, hipEventRecord(c->region_hashed[k], s));
  c->region_keys[k] = d_keys;
  c->region_cur = k;
  c->region_grouped[k] = false;
  return SD_CAS_OK;
}

int sd_cas_group_regions_dev(sd_cas_ctx* c, size_t n, uint32_t* d_rep, uint64_t* out_objects,
                             void* stream) {
  if (!c) return SD_CAS_EINVAL;
  const int k = c->region_cur;
  if (k < 0 || c->region_grouped[k] || c->region_n[k] != n || !d_rep)
    return fail(c, SD_CAS_EINVAL, "group_regions: no ungrouped hash_regions batch of %zu files", n);
  HIP_TRY(c, hipSetDevice(c->device));
  hipStream_t s = pick(c, stream);
  uint64_t *rkeys, *gkeys, *skeys;
  uint32_t *rfile, *gvals, *sfile;
  region_group_layout(c->regions[k].p, n, &rkeys, &rfile, &gkeys, &gvals, &skeys, &sfile);
  uint64_t* obj = region_objects(c, k);
  uint32_t* cur = c->gcursor + REGION_SET_WORDS * k;
  HIP_TRY(c, hipStreamWaitEvent(s, c->region_hashed[k], 0));  // after its K1G, whatever stream
  hipError_t e = region_group_min(rkeys, rfile, cur, region_capacity(n), d_rep, obj, gkeys, gvals,
                                  c->region_keys[k], n, skeys, sfile, s);
  if (e != hipSuccess) {
    (void)hipMemsetAsync(cur, 0, REGION_SET_WORDS * 4, s);
    return fail(c, SD_CAS_EHIP, "group_regions: %s", hipGetErrorString(e));
  }
  HIP_TRY(c, hipEventRecord(c->region_done[k], s));
  c->region_pending[k] = true;
  c->region_grouped[k] = true;
  c->region_obj_set = k;
  if (out_objects) {
    HIP_TRY(c, hipMemcpyAsync(out_objects, obj, 8, hipMemcpyDeviceToHost, s));
    HIP_TRY(c, hipStreamSynchronize(s));
  }
  return SD_CAS_OK;
}

int sd_cas_hash_group_sampled_dev(sd_cas_ctx* c, const void* d_content, uint64_t stride,
                                  const uint64_t* d_sizes, size_t n, uint64_t* d_keys,
                                  uint32_t* d_rep, uint32_t* d_overflow, uint64_t* out_objects,
                                  void* stream) {
  if (!c) return SD_CAS_EINVAL;
  if (n && (!d_rep || !d_overflow))
    return fail(c, SD_CAS_EINVAL, "hash_group_sampled: null rep/overflow");
  if (!fused_eligible(c, n)) {  // the two calls in sequence
    int rc = sd_cas_hash_sampled_dev(c, d_content, stride, d_sizes, n, d_keys, stream);
    if (rc) return rc;
    return sd_cas_group_dev(c, d_keys, n, d_rep, out_objects, stream);
  }
  int rc = sd_cas_hash_regions_sampled_dev(c, d_content, stride, d_sizes, n, d_keys, d_rep,
                                           d_overflow, stream);
  if (rc) return rc;
  // (an overflowed region is regrouped by its own table workgroup: exact either way)
  return sd_cas_group_regions_dev(c, n, d_rep, out_objects, stream);
}

int sd_cas_group_min_dev(sd_cas_ctx* c, const uint64_t* d_keys, const uint32_t* d_vals, size_t n,
                         uint32_t* d_out, uint64_t* out_objects, void* stream) {
  if (!c) return SD_CAS_EINVAL;
  if (n >= (1ull << 32) || (n && (!d_keys || !d_out)))
    return fail(c, SD_CAS_EINVAL, "group_min: bad arguments");
  if (c->group_method == SD_CAS_GROUP_HASH && !hash_group_supported(n))
    return fail(c, SD_CAS_EINVAL, "group_min: %zu keys exceed the hash grouping's range", n);
  hipStream_t s = pick(c, stream);
  if (c->use_hash_group(n)) {
    int rc = ensure(c, c->ws, hash_group_workspace_bytes(n, c->group_target));
    if (rc) return rc;
    HIP_TRY(c, sd_ws_acquire(c, s));
    HIP_TRY(c, hash_group_min(d_keys, d_vals, n, d_out, c->d_scalar, c->ws.p, c->gtotals, s,
                              c->group_target));
  } else {  // beyond the hash grouping's range: stable LSD sort of (key, val) + run minima
    int rc = ensure(c, c->ws, group_min_sorted_workspace_bytes(n));
    if (rc) return rc;
    HIP_TRY(c, sd_ws_acquire(c, s));
    HIP_TRY(c, group_min_by_sort(d_keys, d_vals, n, d_out, c->d_scalar, c->ws.p, s));
  }
  HIP_TRY(c, sd_ws_release(c, s));
  c->region_obj_set = -1;
  if (out_objects) {
    HIP_TRY(c, hipMemcpyAsync(out_objects, c->d_scalar, 8, hipMemcpyDeviceToHost, s));
    HIP_TRY(c, hipStreamSynchronize(s));
  }
  return SD_CAS_OK;
}

int sd_cas_partition_dev(sd_cas_ctx* c, const uint64_t* d_keys, size_t n, uint32_t parts,
                         uint64_t* d_keys_out, uint32_t* d_pos_out, uint64_t* d_counts,
                         void* stream) {
  if (!c) return SD_CAS_EINVAL;
  if (parts == 0 || parts > 16384 || n >= (1ull << 32) || !d_counts ||
      (n && (!d_keys || !d_keys_out || !d_pos_out)))
    return fail(c, SD_CAS_EINVAL, "partition: bad arguments");
  hipStream_t s = pick(c, stream);
  int rc = ensure(c, c->ws, partition_workspace_bytes(n, parts));
  if (rc) return rc;
  HIP_TRY(c, sd_ws_acquire(c, s));
  HIP_TRY(c, partition_range(d_keys, n, parts, d_keys_out, d_pos_out, d_counts, c->ws.p, s));
  HIP_TRY(c, sd_ws_release(c, s));
  return SD_CAS_OK;
}

int sd_cas_group_sorted_dev(sd_cas_ctx* c, const uint64_t* d_sorted_keys,
                            const uint32_t* d_sorted_vals, size_t n, uint32_t* d_rep,
                            uint64_t* out_objects, void* stream) {
  if (!c) return SD_CAS_EINVAL;
  if (n >= (1ull << 32) || (n && (!d_sorted_keys || !d_sorted_vals || !d_rep)))
    return fail(c, SD_CAS_EINVAL, "group_sorted: bad arguments");
  hipStream_t s = pick(c, stream);
  int rc = ensure(c, c->ws, group_workspace_bytes(n));
  if (rc) return rc;
  HIP_TRY(c, sd_ws_acquire(c, s));
  HIP_TRY(c, group_sorted(d_sorted_keys, d_sorted_vals, n, d_rep, c->d_scalar, c->ws.p, s));
  HIP_TRY(c, sd_ws_release(c, s));
  c->region_obj_set = -1;
  if (out_objects) {
    HIP_TRY(c, hipMemcpyAsync(out_objects, c->d_scalar, 8, hipMemcpyDeviceToHost, s));
    HIP_TRY(c, hipStreamSynchronize(s));
  }
  return SD_CAS_OK;
}

int sd_cas_group_chunked_dev(sd_cas_ctx* c, const uint32_t* d_rep, size_t n, uint32_t chunk,
                             uint32_t* d_rep_chunked, uint64_t* out_created,
                             uint64_t* out_linked, void* stream) {
  if (!c) return SD_CAS_EINVAL;
  if (chunk == 0 || n >= (1ull << 32) || (n && (!d_rep || !d_rep_chunked)))
    return fail(c, SD_CAS_EINVAL, "group_chunked: bad arguments");
  hipStream_t s = pick(c, stream);
  uint64_t* d_created = c->d_scalar + 1;
  HIP_TRY(c, sd_ws_acquire(c, s));
  HIP_TRY(c, hipMemsetAsync(d_created, 0, 8, s));
  HIP_TRY(c, group_chunked(d_rep, n, chunk, d_rep_chunked, d_created, s));
  HIP_TRY(c, sd_ws_release(c, s));
  uint64_t created = 0;
  HIP_TRY(c, hipMemcpyAsync(&created, d_created, 8, hipMemcpyDeviceToHost, s));
  HIP_TRY(c, hipStreamSynchronize(s));
  if (out_created) *out_created = created;
  if (out_linked) *out_linked = n - created;
  return SD_CAS_OK;
}

// ---- Object-link emission (file_identifier_job.rs:180-236, mod.rs:98-350) -------------

static_assert(SD_CAS_ROW_HASHED == SD_LINKS_HASHED && SD_CAS_ROW_NO_CAS == SD_LINKS_NO_CAS &&
                  SD_CAS_ROW_ERROR == SD_LINKS_ERROR && SD_CAS_LINK_CREATED == SD_LINKS_CREATED &&
                  SD_CAS_LINK_LINKED == SD_LINKS_LINKED && SD_CAS_LINK_DROPPED == SD_LINKS_DROPPED &&
                  SD_CAS_LINK_NOT_REACHED == SD_LINKS_NOT_REACHED &&
                  SD_CAS_LINK_EXISTING == SD_LINKS_EXISTING &&
                  SD_CAS_NO_STEP == SD_LINKS_NO_STEP && SD_CAS_NO_OBJECT == SD_LINKS_NO_OBJECT,
              "link constants");

size_t sd_cas_identifier_max_steps(size_t n, uint32_t chunk) {
  return chunk ? (n + chunk - 1) / chunk : 0;
}

int sd_cas_identifier_links_seeded_dev(sd_cas_ctx* c, const uint64_t* d_keys, const uint8_t* d_state,
                                       size_t n, uint32_t chunk, const uint64_t* d_seed_keys,
                                       const uint32_t* d_seed_objects, size_t n_seed, uint32_t* d_step,
                                       uint32_t* d_object, uint8_t* d_action, uint64_t* h_step_counts,
                                       size_t max_steps, uint64_t* out_steps, void* stream) {
  if (!c) return SD_CAS_EINVAL;
  const size_t steps_total = sd_cas_identifier_max_steps(n, chunk);
  if (chunk == 0 || n >= (1ull << 32) || !out_steps || max_steps < steps_total ||
      (n && (!d_keys || !d_step || !d_object || !d_action || !h_step_counts)) ||
      (n_seed && (!d_seed_keys || !d_seed_objects)))
    return fail(c, SD_CAS_EINVAL, "identifier_links: bad arguments");
  // a seeded grouping tags rows with LINKS_ROW_FLAG: rows and Object ids below 2^31
  if (n_seed && (n >= LINKS_ROW_FLAG || n_seed >= LINKS_ROW_FLAG || n + n_seed >= (1ull << 32)))
    return fail(c, SD_CAS_EINVAL, "identifier_links: %zu rows + %zu existing Objects exceed 2^31",
                n, n_seed);
  *out_steps = 0;
  for (size_t k = 0; k < 2 * steps_total; k++) h_step_counts[k] = 0;
  if (n == 0) return SD_CAS_OK;
  hipStream_t s = pick(c, stream);
  const bool seeded = n_seed > 0;
  // staging (this call is blocking): rep | hkeys | hrows | minrow | orphans | starts | counts |
  // 2 counters; the seeded grouping runs over the hashed rows + the existing Objects' keys
  const size_t m = n + n_seed;
  const size_t b_rep = up256(n * 4), b_hk = up256(m * 8), b_hr = up256(m * 4), b_mr = up256(m * 4),
               b_or = up256(n * 8), b_st = up256((steps_total + 1) * 4), b_ct = up256(steps_total * 8);
  int rc = ensure(c, c->staging, b_rep + b_hk + b_hr + b_mr + b_or + b_st + b_ct + 256);
  if (rc) return rc;
  char* p = (char*)c->staging.p;
  uint32_t* rep = (uint32_t*)p; p += b_rep;
  uint64_t* hkeys = (uint64_t*)p; p += b_hk;
  uint32_t* hrows = (uint32_t*)p; p += b_hr;
  uint32_t* minrow = (uint32_t*)p; p += b_mr;
  uint64_t* orphans = (uint64_t*)p; p += b_or;
  uint32_t* starts = (uint32_t*)p; p += b_st;
  uint32_t* counts = (uint32_t*)p; p += b_ct;
  uint64_t* counters = (uint64_t*)p;
  // 1. grouping over the hashed rows (rep = the key's first row; seeded: the lowest existing
  //    Object id when the key has one — mod.rs:180-198 finds Objects by cas over the whole
  //    library), and the rows that stay orphan after being processed (they steer the cursor)
  std::vector<uint64_t> stay;  // row << 8 | state, ascending
  if (d_state || seeded) {
    uint64_t cnt[2] = {0, 0};
    HIP_TRY(c, hipMemsetAsync(counters, 0, 16, s));
    HIP_TRY(c, links_split(d_keys, d_state, n, hkeys, hrows, counters, orphans, counters + 1,
                           seeded ? LINKS_ROW_FLAG : 0u, s));
    HIP_TRY(c, hipMemcpyAsync(cnt, counters, 16, hipMemcpyDeviceToHost, s));
    HIP_TRY(c, hipStreamSynchronize(s));
    stay.resize(cnt[1]);
    if (cnt[1]) {
      HIP_TRY(c, hipMemcpyAsync(stay.data(), orphans, cnt[1] * 8, hipMemcpyDeviceToHost, s));
    }
    if (seeded) {  // the existing Objects' (cas key, id) pairs after the hashed rows
      HIP_TRY(c, hipMemcpyAsync(hkeys + cnt[0], d_seed_keys, n_seed * 8, hipMemcpyDeviceToDevice, s));
      HIP_TRY(c, hipMemcpyAsync(hrows + cnt[0], d_seed_objects, n_seed * 4, hipMemcpyDeviceToDevice, s));
    }
    if (cnt[0]) {
      if ((rc = sd_cas_group_min_dev(c, hkeys, hrows, cnt[0] + n_seed, minrow, nullptr, s))) return rc;
      HIP_TRY(c, links_scatter(minrow, hrows, cnt[0], rep, seeded ? LINKS_ROW_FLAG : 0u, s));
    }
    HIP_TRY(c, hipStreamSynchronize(s));
    std::sort(stay.begin(), stay.end());
  } else {
    if ((rc = sd_cas_group_dev(c, d_keys, n, rep, nullptr, s))) return rc;
  }
  // 2. the cursor walk (host; O(steps + orphans)): step k covers [start, start + chunk);
  //    the next cursor is its last row, which the next query returns again iff it is
  //    still orphan; an empty query ends the job
  // the rows asked about only increase (each step's last row), so one forward pointer into
  // the sorted orphan list answers them all: O(steps + orphans) (a binary search per step
  // cost ~2 ms of a 10 M-row job)
  size_t sp = 0;
  auto stays = [&](uint64_t row, uint8_t* st) {
    while (sp < stay.size() && (stay[sp] >> 8) < row) ++sp;
    if (sp == stay.size() || (stay[sp] >> 8) != row) return false;
    *st = (uint8_t)(stay[sp] & 0xFF);
    return true;
  };
  std::vector<uint32_t> h_starts;
  h_starts.reserve(steps_total + 1);
  std::vector<uint64_t> extra(steps_total, 0);  // re-queried empty rows: one creation per step
  uint64_t start = 0, reached = 0;
  for (size_t k = 0; k < steps_total && start < n; k++) {
    h_starts.push_back((uint32_t)start);
    const uint64_t end = std::min<uint64_t>(start + chunk, n), last = end - 1;
    reached = end;
    uint8_t st = 0;
    if (stays(last, &st)) {
      if (st == SD_CAS_ROW_NO_CAS && k + 1 < steps_total) extra[k] += 1;
      start = last;
    } else {
      start = end;
    }
  }
  const size_t nsteps = h_starts.size();
  h_starts.push_back(0xFFFFFFFFu);  // sentinel
  // 3. per-row decisions + per-step counts (device)
  HIP_TRY(c, hipMemcpyAsync(starts, h_starts.data(), h_starts.size() * 4, hipMemcpyHostToDevice, s));
  HIP_TRY(c, hipMemsetAsync(counts, 0, std::max<size_t>(nsteps, 1) * 8, s));
  HIP_TRY(c, links_decide(d_state, rep, n, starts, (uint32_t)nsteps, reached, d_step, d_object,
                          d_action, counts, seeded, s));
  std::vector<uint32_t> hc(2 * std::max<size_t>(nsteps, 1));
  HIP_TRY(c, hipMemcpyAsync(hc.data(), counts, hc.size() * 4, hipMemcpyDeviceToHost, s));
  HIP_TRY(c, hipStreamSynchronize(s));
  for (size_t k = 0; k < nsteps; k++) {
    h_step_counts[2 * k] = hc[2 * k] + extra[k];
    h_step_counts[2 * k + 1] = hc[2 * k + 1];
  }
  *out_steps = nsteps;
  return SD_CAS_OK;
}

int sd_cas_identifier_links_dev(sd_cas_ctx* c, const uint64_t* d_keys, const uint8_t* d_state,
                                size_t n, uint32_t chunk, uint32_t* d_step, uint32_t* d_object,
                                uint8_t* d_action, uint64_t* h_step_counts, size_t max_steps,
                                uint64_t* out_steps, void* stream) {
  return sd_cas_identifier_links_seeded_dev(c, d_keys, d_state, n, chunk, nullptr, nullptr, 0, d_step,
                                            d_object, d_action, h_step_counts, max_steps, out_steps,
                                            stream);
}

int sd_cas_identifier_links_seeded(sd_cas_ctx* c, const uint64_t* h_keys, const uint8_t* h_state,
                                   size_t n, uint32_t chunk, const uint64_t* h_seed_keys,
                                   const uint32_t* h_seed_objects, size_t n_seed, uint32_t* h_step,
                                   uint32_t* h_object, uint8_t* h_action, uint64_t* h_step_counts,
                                   size_t max_steps, uint64_t* out_steps) {
  if (!c) return SD_CAS_EINVAL;
  if ((n && (!h_keys || !h_step || !h_object || !h_action)) ||
      (n_seed && (!h_seed_keys || !h_seed_objects)))
    return fail(c, SD_CAS_EINVAL, "identifier_links: bad arguments");
  for (size_t j = 0; j < n_seed; j++)
    if (h_seed_objects[j] >= LINKS_ROW_FLAG)
      return fail(c, SD_CAS_EINVAL, "identifier_links: existing Object id %u >= 2^31", h_seed_objects[j]);
  if (n == 0 || n >= (1ull << 32))
    return sd_cas_identifier_links_dev(c, nullptr, nullptr, n, chunk, nullptr, nullptr, nullptr,
                                       h_step_counts, max_steps, out_steps, c->stream);
  HIP_TRY(c, hipSetDevice(c->device));
  // device copies (c->io): keys | state | step | object | action | seed keys | seed ids
  const size_t bk = up256(n * 8), bs = up256(n), b4 = up256(n * 4);
  const size_t bsk = up256(n_seed * 8), bso = up256(n_seed * 4);
  int rc = ensure(c, c->io, bk + 2 * bs + 2 * b4 + bsk + bso);
  if (rc) return rc;
  char* p = (char*)c->io.p;
  uint64_t* d_keys = (uint64_t*)p; p += bk;
  uint8_t* d_state = h_state ? (uint8_t*)p : nullptr; p += bs;
  uint32_t* d_step = (uint32_t*)p; p += b4;
  uint32_t* d_object = (uint32_t*)p; p += b4;
  uint8_t* d_action = (uint8_t*)p; p += bs;
  uint64_t* d_seed_keys = (uint64_t*)p; p += bsk;
  uint32_t* d_seed_objects = (uint32_t*)p;
  hipStream_t s = c->stream;
  HIP_TRY(c, hipMemcpyAsync(d_keys, h_keys, n * 8, hipMemcpyHostToDevice, s));
  if (h_state) HIP_TRY(c, hipMemcpyAsync(d_state, h_state, n, hipMemcpyHostToDevice, s));
  if (n_seed) {
    HIP_TRY(c, hipMemcpyAsync(d_seed_keys, h_seed_keys, n_seed * 8, hipMemcpyHostToDevice, s));
    HIP_TRY(c, hipMemcpyAsync(d_seed_objects, h_seed_objects, n_seed * 4, hipMemcpyHostToDevice, s));
  }
  rc = sd_cas_identifier_links_seeded_dev(c, d_keys, d_state, n, chunk, d_seed_keys, d_seed_objects,
                                          n_seed, d_step, d_object, d_action, h_step_counts,
                                          max_steps, out_steps, s);
  if (rc) return rc;
  HIP_TRY(c, hipMemcpyAsync(h_step, d_step, n * 4, hipMemcpyDeviceToHost, s));
  HIP_TRY(c, hipMemcpyAsync(h_object, d_object, n * 4, hipMemcpyDeviceToHost, s));
  HIP_TRY(c, hipMemcpyAsync(h_action, d_action, n, hipMemcpyDeviceToHost, s));
  HIP_TRY(c, hipStreamSynchronize(s));
  return SD_CAS_OK;
}

int sd_cas_identifier_links(sd_cas_ctx* c, const uint64_t* h_keys, const uint8_t* h_state,
                            size_t n, uint32_t chunk, uint32_t* h_step, uint32_t* h_object,
                            uint8_t* h_action, uint64_t* h_step_counts, size_t max_steps,
                            uint64_t* out_steps) {
  return sd_cas_identifier_links_seeded(c, h_keys, h_state, n, chunk, nullptr, nullptr, 0, h_step,
                                        h_object, h_action, h_step_counts, max_steps, out_steps);
}

// ---- host-buffer cas (blocking) -----------------------------------------------------

// Stage layout in pinned memory and on the device:
//   [sampled contents, 57,344 B each, contiguous] [packed contents, 128-B aligned]
//   [sizes_s u64][sizes_p u64][offs_p u64][lens_p u32]   (small metadata)
struct Plan {
  std::vector<size_t> sampled, packed;  // file indices
  std::vector<uint64_t> poff;           // packed offsets (relative to packed base)
  size_t sampled_bytes = 0, packed_bytes = 0;
};

static int plan_batch(sd_cas_ctx* c, const uint64_t* buf_lens, const uint64_t* sizes, size_t n,
                      Plan& pl) {
  for (size_t i = 0; i < n; i++) {
    if (sizes[i] > MINIMUM_FILE_SIZE) {
      if (buf_lens[i] != SAMPLED_CONTENT_LEN)
        return fail(c, SD_CAS_EINVAL, "file %zu: size %llu > %llu needs %u sampled bytes, got %llu",
                    i, (unsigned long long)sizes[i], (unsigned long long)MINIMUM_FILE_SIZE,
                    SAMPLED_CONTENT_LEN, (unsigned long long)buf_lens[i]);
      pl.sampled.push_back(i);
    } else {
      if (buf_lens[i] > MAX_PACKED_CONTENT_LEN)
        return fail(c, SD_CAS_EINVAL, "file %zu: whole-file content %llu exceeds %u", i,
                    (unsigned long long)buf_lens[i], MAX_PACKED_CONTENT_LEN);
      pl.packed.push_back(i);
      pl.poff.push_back(pl.packed_bytes);
      pl.packed_bytes += up128(buf_lens[i]);
    }
  }
  pl.sampled_bytes = pl.sampled.size() * (size_t)SAMPLED_CONTENT_LEN;
  pl.packed_bytes += 16;  // tail pad
  return SD_CAS_OK;
}

// Host side of a staged batch's metadata (sizes of both sub-batches, packed offsets; the
// packed lens are written by the caller): [content][sizes][poffs][plens][keys].
static void stage_meta(const Plan& pl, const uint64_t* sizes, char* pin) {
  const size_t ns = pl.sampled.size(), np = pl.packed.size();
  const size_t content_bytes = pl.sampled_bytes + up256(pl.packed_bytes);
  uint64_t* h_sizes = (uint64_t*)(pin + content_bytes);
  uint64_t* h_poffs = (uint64_t*)((char*)h_sizes + up256((ns + np) * 8));
  for (size_t k = 0; k < ns; k++) h_sizes[k] = sizes[pl.sampled[k]];
  for (size_t k = 0; k < np; k++) h_sizes[ns + k] = sizes[pl.packed[k]];
  for (size_t k = 0; k < np; k++) h_poffs[k] = pl.poff[k];
}

// The kernels of a host batch write its keys straight into the pinned staging (at the
// staging's keys offset) instead of HBM + a D2H copy: a few KiB of posted writes over the
// host link, and one fewer copy in the call's serial tail (SD_PATHS_KEYS_TO_HOST, A/B)
#ifndef SD_PATHS_KEYS_TO_HOST
#define SD_PATHS_KEYS_TO_HOST 1
#endif

// byte offset of the keys in a staged batch: content | sizes | poffs | plens | keys
static size_t staged_keys_offset(const Plan& pl) {
  const size_t ns = pl.sampled.size(), np = pl.packed.size();
  return pl.sampled_bytes + up256(pl.packed_bytes) + up256((ns + np) * 8) + up256(np * 8) + up256(np * 4);
}

// Enqueues, for a batch staged in pinned memory at `pin` (stage_meta done): H2D of
// [h2d_lo, h2d_hi) of the staging to `dev` on the copy stream (the rest is already there),
// both hash sub-batches on the compute stream after it, their keys into `pin`'s keys area
// (scatter_keys reads them there).  `done` (optional) is recorded on the compute stream after it.
// The device-side views of a staged batch: content | sizes | poffs | plens, keys in `pin`
// (SD_PATHS_KEYS_TO_HOST) or on the device.
struct StagedDev {
  uint64_t* sizes;
  uint64_t* poffs;
  uint32_t* plens;
  uint64_t* keys;
};
static StagedDev staged_dev(const Plan& pl, char* pin, char* dev) {
  const size_t ns = pl.sampled.size(), np = pl.packed.size();
  const size_t content_bytes = pl.sampled_bytes + up256(pl.packed_bytes);
  StagedDev d;
  d.sizes = (uint64_t*)(dev + content_bytes);
  d.poffs = (uint64_t*)((char*)d.sizes + up256((ns + np) * 8));
  d.plens = (uint32_t*)((char*)d.poffs + up256(np * 8));
  d.keys = (uint64_t*)((SD_PATHS_KEYS_TO_HOST ? pin : dev) + staged_keys_offset(pl));
  return d;
}

// the whole-file sub-batch's hash on stream s (K1L at job-step sizes)
static int enqueue_packed(sd_cas_ctx* c, const Plan& pl, char* pin, char* dev, hipStream_t s) {
  const size_t ns = pl.sampled.size(), np = pl.packed.size();
  const StagedDev d = staged_dev(pl, pin, dev);
  return np ? sd_cas_hash_packed_dev(c, dev + pl.sampled_bytes, d.poffs, d.plens, d.sizes + ns, np,
                                     d.keys + ns, s)
            : SD_CAS_OK;
}

static int enqueue_hash(sd_cas_ctx* c, const Plan& pl, size_t n, char* pin, char* dev,
                        hipEvent_t done, size_t h2d_lo, size_t h2d_hi, bool packed_enqueued = false) {
  const size_t ns = pl.sampled.size();
  const StagedDev d = staged_dev(pl, pin, dev);
  (void)n;
  if (h2d_hi > h2d_lo)
    HIP_TRY(c, hipMemcpyAsync(dev + h2d_lo, pin + h2d_lo, h2d_hi - h2d_lo, hipMemcpyHostToDevice, c->copy));
  HIP_TRY(c, hipEventRecord(c->h2d_done, c->copy));
  HIP_TRY(c, hipStreamWaitEvent(c->stream, c->h2d_done, 0));
  int rc;
  if (ns && (rc = sd_cas_hash_sampled_dev(c, dev, SAMPLED_CONTENT_LEN, d.sizes, ns, d.keys,
                                          c->stream)))
    return rc;
  if (!packed_enqueued && (rc = enqueue_packed(c, pl, pin, dev, c->stream))) return rc;
  // an early whole-file hash ran on copy2, beside the sampled one: join it
  if (packed_enqueued) HIP_TRY(c, hipStreamWaitEvent(c->stream, c->packed_done, 0));
  if (!SD_PATHS_KEYS_TO_HOST)
    HIP_TRY(c, hipMemcpyAsync(pin + staged_keys_offset(pl), d.keys,
                              (ns + pl.packed.size()) * 8, hipMemcpyDeviceToHost, c->stream));
  if (done) HIP_TRY(c, hipEventRecord(done, c->stream));
  return SD_CAS_OK;
}

// bytes of the staging before its keys: content + sizes + poffs + plens
static size_t staged_h2d_bytes(const Plan& pl) {
  const size_t ns = pl.sampled.size(), np = pl.packed.size();
  return pl.sampled_bytes + up256(pl.packed_bytes) + up256((ns + np) * 8) + up256(np * 8) + up256(np * 4);
}

static int enqueue_staged(sd_cas_ctx* c, const Plan& pl, const uint64_t* sizes, size_t n,
                          char* pin, char* dev, hipEvent_t done) {
  stage_meta(pl, sizes, pin);
  return enqueue_hash(c, pl, n, pin, dev, done, 0, staged_h2d_bytes(pl));
}

static void scatter_keys(const Plan& pl, const char* pin, uint64_t* out_keys) {
  const uint64_t* h_keys = (const uint64_t*)(pin + staged_keys_offset(pl));
  const size_t ns = pl.sampled.size(), np = pl.packed.size();
  for (size_t k = 0; k < ns; k++) out_keys[pl.sampled[k]] = h_keys[k];
  for (size_t k = 0; k < np; k++) out_keys[pl.packed[k]] = h_keys[ns + k];
}

static size_t staged_pinned_bytes(const Plan& pl, size_t n);

// One staged batch, blocking: staging at c->pinned, device copy in c->staging.
static int run_staged(sd_cas_ctx* c, const Plan& pl, const uint64_t* sizes, size_t n,
                      uint64_t* out_keys) {
  int rc = ensure(c, c->staging, staged_pinned_bytes(pl, n));
  if (rc) return rc;
  if ((rc = enqueue_staged(c, pl, sizes, n, (char*)c->pinned, (char*)c->staging.p, nullptr)))
    return rc;
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  scatter_keys(pl, (const char*)c->pinned, out_keys);
  return SD_CAS_OK;
}

static size_t staged_pinned_bytes(const Plan& pl, size_t n) {
  const size_t ns = pl.sampled.size(), np = pl.packed.size();
  return pl.sampled_bytes + up256(pl.packed_bytes) + up256((ns + np) * 8) + up256(np * 8) +
         up256(np * 4) + up256(n * 8);
}

int sd_cas_generate_cas_ids(sd_cas_ctx* c, const uint8_t* const* bufs, const uint64_t* buf_lens,
                            const uint64_t* sizes, size_t n, uint64_t* out_keys) {
  if (!c) return SD_CAS_EINVAL;
  if (n == 0) return SD_CAS_OK;
  if (!bufs || !buf_lens || !sizes || !out_keys || n >= (1ull << 32))
    return fail(c, SD_CAS_EINVAL, "generate_cas_ids: null argument");
  HIP_TRY(c, hipSetDevice(c->device));
  Plan pl;
  int rc = plan_batch(c, buf_lens, sizes, n, pl);
  if (rc) return rc;
  rc = ensure_pinned(c, staged_pinned_bytes(pl, n));
  if (rc) return rc;
  char* pin = (char*)c->pinned;
  for (size_t k = 0; k < pl.sampled.size(); k++)
    memcpy(pin + k * (size_t)SAMPLED_CONTENT_LEN, bufs[pl.sampled[k]], SAMPLED_CONTENT_LEN);
  char* pbase = pin + pl.sampled_bytes;
  const size_t ns = pl.sampled.size(), np = pl.packed.size();
  const size_t content_bytes = pl.sampled_bytes + up256(pl.packed_bytes);
  uint32_t* h_plens = (uint32_t*)(pin + content_bytes + up256((ns + np) * 8) + up256(np * 8));
  for (size_t k = 0; k < np; k++) {
    const size_t i = pl.packed[k];
    if (buf_lens[i]) memcpy(pbase + pl.poff[k], bufs[i], buf_lens[i]);
    h_plens[k] = (uint32_t)buf_lens[i];
  }
  return run_staged(c, pl, sizes, n, out_keys);
}

static int cas_ids_from_paths(sd_cas_ctx* c, const char* const* paths, const uint64_t* sizes,
                              size_t n, uint64_t* out_keys, int32_t* status, uint64_t* out_sizes);

int sd_cas_generate_cas_ids_from_paths(sd_cas_ctx* c, const char* const* paths,
                                       const uint64_t* sizes, size_t n, uint64_t* out_keys,
                                       int32_t* status) {
  return cas_ids_from_paths(c, paths, sizes, n, out_keys, status, nullptr);
}

int sd_cas_file_metadata_from_paths(sd_cas_ctx* c, const char* const* paths, size_t n,
                                    uint64_t* out_keys, int32_t* status, uint64_t* out_sizes) {
  if (c && n && !out_sizes) return fail(c, SD_CAS_EINVAL, "file_metadata_from_paths: null out_sizes");
  return cas_ids_from_paths(c, paths, nullptr, n, out_keys, status, out_sizes);
}

static int cas_ids_from_paths(sd_cas_ctx* c, const char* const* paths, const uint64_t* sizes,
                              size_t n, uint64_t* out_keys, int32_t* status, uint64_t* out_sizes) {
  if (!c) return SD_CAS_EINVAL;
  if (n == 0) return SD_CAS_OK;
  if (!paths || !out_keys || !status || n >= (1ull << 32))
    return fail(c, SD_CAS_EINVAL, "generate_cas_ids_from_paths: null argument");
  SdTrace tr(c->trace, "from_paths", n);
  HIP_TRY(c, hipSetDevice(c->device));
  for (size_t i = 0; i < n; i++) {
    status[i] = 0;
    out_keys[i] = 0;
  }
  // FileMetadata::new (file_identifier/mod.rs:63-86): the metadata — given by the caller, or
  // taken here with stat (fs::metadata follows symlinks) — decides the row: an error drops
  // it (-errno), a directory is refused (-EISDIR; the reference asserts, :67-70), length 0
  // means no cas_id (SD_CAS_STATUS_NO_CAS, nothing is read: :78-86), anything else is
  // generate_cas_id(path, len).
  std::vector<uint64_t> msize;
  if (!sizes) {
    msize.assign(n, 0);
    std::atomic<size_t> next{0};
    c->pool.run(std::max(1u, std::min(16u, (unsigned)((n + 63) / 64))), [&]() {
      for (size_t i; (i = next.fetch_add(1)) < n;) {
        struct stat st;
        if (stat(paths[i], &st) != 0) { status[i] = -errno; continue; }
        if (S_ISDIR(st.st_mode)) { status[i] = -EISDIR; continue; }
        msize[i] = (uint64_t)st.st_size;
      }
    });
    sizes = msize.data();
    tr.mark("stat");
  }
  if (out_sizes) std::copy(sizes, sizes + n, out_sizes);
  for (size_t i = 0; i < n; i++)
    if (status[i] == 0 && sizes[i] == 0) status[i] = SD_CAS_STATUS_NO_CAS;
  // Content length per file: sampled 57,344; whole file = its actual length (cas.rs:29
  // reads the file, not `size` bytes).  The plan assumes the actual length is `size` (the
  // metadata just read, mod.rs:63,78-79); the gather checks it with fstat on the open
  // descriptor — no second path walk — and a whole file whose length changed is re-read and
  // hashed after the windows (`redo`).  Rows already decided (error, no cas) plan as empty
  // whole files and are never read.
  std::vector<uint64_t> lens(n, 0);
  std::vector<uint8_t> redo(n, 0);
  for (size_t i = 0; i < n; i++)
    lens[i] = status[i] ? 0 : sizes[i] > MINIMUM_FILE_SIZE ? SAMPLED_CONTENT_LEN : sizes[i];
  // Windows of files, double-buffered: the pool gathers window w into one pinned slot while
  // the GPU copies and hashes window w-1 from the other.  The call takes about (gather of all
  // windows) + (H2D + hash of the last one), so windows are cut by staged BYTES — about a
  // twelfth of the batch each (2-64 MiB, <= GATHER_WINDOW files): config 1's 10k tmpfs files
  // (~40 KB staged each) run in ~12 windows of ~830 files instead of 5 of 2,048, and the
  // un-overlapped tail shrinks with the last window.  A batch whose whole gather is shorter
  // than what a second window's launch chain costs — the reference's 100-file job step
  // (mod.rs:34), up to SMALL_BATCH_FILES files and SMALL_BATCH_BYTES staged — is one window:
  // cutting its ~4 MB in two added a second H2D/hash/D2H chain and its serial tail
  // (0.36-0.41 -> 0.48-0.52 ms per step).
  constexpr size_t GATHER_WINDOW = 2048;
  constexpr size_t SMALL_BATCH_FILES = 2048;
  constexpr uint64_t SMALL_BATCH_BYTES = 16ull << 20;
  std::vector<size_t> wstart{0};
  {
    uint64_t total = 0;
    for (size_t i = 0; i < n; i++) total += up128(lens[i]);
    const bool one_window = n <= SMALL_BATCH_FILES && total <= SMALL_BATCH_BYTES;
    const uint64_t target = one_window ? SMALL_BATCH_BYTES
                                       : std::min<uint64_t>(64ull << 20, std::max<uint64_t>(2ull << 20, total / 12));
    uint64_t bytes = 0;
    for (size_t i = 0; i < n; i++) {
      const size_t files = i - wstart.back();
      if (files && (files == GATHER_WINDOW || bytes + up128(lens[i]) > target)) {
        wstart.push_back(i);
        bytes = 0;
      }
      bytes += up128(lens[i]);
    }
    wstart.push_back(n);
  }
  const size_t nw = wstart.size() - 1;
  std::vector<Plan> plans(nw);
  size_t slot = 0;
  // decided rows plan as empty whole files (their metadata size may be anything)
  std::vector<uint64_t> psize(sizes, sizes + n);
  for (size_t i = 0; i < n; i++)
    if (status[i]) psize[i] = 0;
  for (size_t w = 0; w < nw; w++) {
    const size_t f0 = wstart[w], m = wstart[w + 1] - wstart[w];
    int rc = plan_batch(c, lens.data() + f0, psize.data() + f0, m, plans[w]);
    if (rc) return rc;
    slot = std::max(slot, up256(staged_pinned_bytes(plans[w], m)));
  }
  const int nslots = nw > 1 ? 2 : 1;
  int rc = ensure_pinned(c, nslots * slot);
  if (rc) return rc;
  if ((rc = ensure(c, c->staging, nslots * slot))) return rc;
  hipEvent_t* done = c->gather_done;
  tr.mark("plan");
  // The single-window batch (up to SMALL_BATCH_FILES: the reference's 100-file job step)
  // streams its H2D behind the gather instead of after it: the pool threads read the files
  // while this thread copies each finished prefix of the staging (STREAM_CHUNK bytes or
  // more at a time) on the copy stream, so the batch costs about max(gather, H2D) + the last
  // piece + the hash, not gather + H2D + hash.
#ifndef SD_PATHS_ZERO_COPY
#define SD_PATHS_ZERO_COPY 0
#endif
#ifndef SD_PATHS_STREAM_CHUNK_KB
#define SD_PATHS_STREAM_CHUNK_KB 512
#endif
#ifndef SD_PATHS_COPY_STREAMS
#define SD_PATHS_COPY_STREAMS 1  // 2: the pieces alternate between two copy streams (A/B)
#endif
#ifndef SD_PATHS_PULL
#define SD_PATHS_PULL 1  // the pieces are copied by a kernel (sd_pull_host), not the SDMA engine
#endif
#ifndef SD_PATHS_FIRST_KB
#define SD_PATHS_FIRST_KB 128
#endif
#ifndef SD_PATHS_RAMP
#define SD_PATHS_RAMP 0
#endif
// A streamed batch with both kinds of file reads and sends its whole files FIRST and hashes
// them as soon as they have landed, while the sampled files' pieces still cross the link:
// the whole-file K1L (up to 101 chunks: 2 chunks per lane, ~58 us) then overlaps the
// transfer instead of running after the sampled K1L (~35 us) at the end of the step.
#ifndef SD_PATHS_PACKED_FIRST
#define SD_PATHS_PACKED_FIRST 1
#endif
  constexpr size_t STREAM_CHUNK = (size_t)SD_PATHS_STREAM_CHUNK_KB << 10;
  constexpr size_t STREAM_FIRST = (size_t)SD_PATHS_FIRST_KB << 10;
  constexpr size_t STREAM_MIN_FILES = 16;
  char* pin0 = (char*)c->pinned;
  char* dev0 = (char*)c->staging.p;
  bool packed_early = false;  // the streamed batch's whole-file hash is already enqueued
  auto gather = [&](size_t w, char* pin, char* dev, bool streamed) {
    const Plan& pl = plans[w];
    const size_t f0 = wstart[w], m = wstart[w + 1] - wstart[w];
    const size_t ns = pl.sampled.size(), np = pl.packed.size();
    const size_t content_bytes = pl.sampled_bytes + up256(pl.packed_bytes);
    uint32_t* h_plens = (uint32_t*)(pin + content_bytes + up256((ns + np) * 8) + up256(np * 8));
    for (size_t k = 0; k < np; k++) h_plens[k] = (uint32_t)lens[f0 + pl.packed[k]];
    const size_t items = ns + np;
    // visit order (streamed, both kinds present): the whole files, then the sampled ones;
    // staging item t of visit slot v, and fin[] indexed by v
    const bool packed_first = streamed && SD_PATHS_PACKED_FIRST && ns > 0 && np > 0;
    auto vis = [&](size_t v) -> size_t { return !packed_first ? v : v < np ? ns + v : v - np; };
    packed_early = false;
    std::atomic<size_t> next{0};
    std::unique_ptr<std::atomic<uint8_t>[]> fin;
    if (streamed) {
      fin.reset(new std::atomic<uint8_t>[items]);
      for (size_t t = 0; t < items; t++) fin[t].store(0, std::memory_order_relaxed);
    }
    auto item = [&](size_t t) {
        const size_t li = t < ns ? pl.sampled[t] : pl.packed[t - ns];
        const size_t i = f0 + li;
        if (status[i]) return;
        char* dst = t < ns ? pin + t * (size_t)SAMPLED_CONTENT_LEN
                           : pin + pl.sampled_bytes + pl.poff[t - ns];
        int fd = open(paths[i], O_RDONLY | O_CLOEXEC);
        if (fd < 0) { status[i] = -errno; return; }
        // a whole file is checked against its metadata length here; a sampled file needs no
        // fstat before its reads (a directory's pread fails with EISDIR, the same status)
        if (sizes[i] <= MINIMUM_FILE_SIZE) {
          struct stat st;
          if (fstat(fd, &st) != 0) { status[i] = -errno; close(fd); return; }
          if (S_ISDIR(st.st_mode)) { status[i] = -EISDIR; close(fd); return; }
          if ((uint64_t)st.st_size != lens[i]) {
            redo[i] = 1;
            close(fd);
            return;
          }
        }
        // cas.rs:35-58 offsets: header at 0, sample k at 8192 + k*jump (both from `size`,
        // the metadata length), footer at the file's ACTUAL end - 8192: the reference
        // seeks SeekFrom::End(-8192) (cas.rs:54-55), so it is located after the samples
        // with fstat on the open descriptor (a grown or shrunk file keeps the reference's
        // outcome: a cas_id while every read fits, UnexpectedEof = -EIO otherwise)
        // the header and sample 0 are contiguous in the file ([0, 8192) and [8192, 18432):
        // the first sample is read where the header read left off, cas.rs:35-44), so they
        // are one pread — the outcome of a short file is the same UnexpectedEof either way
        uint64_t offs[5], lns[5];
        int parts;
        const bool sampled = sizes[i] > MINIMUM_FILE_SIZE;
        if (sampled) {
          const uint64_t jump = (sizes[i] - 2 * HEADER_OR_FOOTER_SIZE) / SAMPLE_COUNT;
          offs[0] = 0; lns[0] = HEADER_OR_FOOTER_SIZE + SAMPLE_SIZE;
          for (int k = 1; k < 4; k++) { offs[k] = HEADER_OR_FOOTER_SIZE + k * jump; lns[k] = SAMPLE_SIZE; }
          offs[4] = 0; lns[4] = HEADER_OR_FOOTER_SIZE;  // offset set below
          parts = 5;
        } else {
          offs[0] = 0; lns[0] = lens[i];
          parts = 1;
        }
        for (int k = 0; k < parts && !status[i] && !redo[i]; k++) {
          if (sampled && k == 4) {
            struct stat st;
            if (fstat(fd, &st) != 0) { status[i] = -errno; break; }
            // lseek to a negative position: EINVAL (io::ErrorKind::InvalidInput)
            if ((uint64_t)st.st_size < HEADER_OR_FOOTER_SIZE) { status[i] = -EINVAL; break; }
            offs[4] = (uint64_t)st.st_size - HEADER_OR_FOOTER_SIZE;
          }
          size_t got = 0;
          while (got < lns[k]) {
            ssize_t r = pread(fd, dst + got, lns[k] - got, (off_t)(offs[k] + got));
            if (r < 0) { if (errno == EINTR) continue; status[i] = -errno; break; }
            if (r == 0) {  // sampled: UnexpectedEof; whole file: it shrank after fstat
              if (sizes[i] > MINIMUM_FILE_SIZE) status[i] = -EIO; else redo[i] = 1;
              break;
            }
            got += (size_t)r;
          }
          dst += lns[k];
        }
        close(fd);
    };
    auto worker = [&]() {
      for (size_t v; (v = next.fetch_add(1)) < items;) {
        item(vis(v));
        if (streamed) fin[v].store(1, std::memory_order_release);
      }
    };
    if (!streamed) {
      c->pool.run(std::max(1u, std::min(16u, (unsigned)((m + 7) / 8))), worker);
      return SD_CAS_OK;
    }
    // streamed: this thread pumps the copies, up to 15 pool threads read (~7 files each for
    // a 100-file step; the job's share of the host is 16 cores)
    const unsigned threads = std::max(1u, std::min(15u, (unsigned)((m + 6) / 7)));
    // the pump: metadata first, then each finished prefix of the content (items are taken
    // in staging order, so a prefix of items is a prefix of bytes)
    int prc = SD_CAS_OK;
    size_t ncopies = 0, ncopies_all = 0, npieces = 0;
    double copy_us = 0, first_us = -1, last_us = 0;
    const auto t_pump = std::chrono::steady_clock::now();
    auto since = [&](std::chrono::steady_clock::time_point a) {
      return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - a).count();
    };
    // the pump works in a VIRTUAL byte space laid out in visit order — with packed_first,
    // [whole-file area (P bytes, incl. its tail pad)][sampled area] — mapped back to the
    // staging's [sampled][whole-file] layout by phys()
    const size_t P = content_bytes - pl.sampled_bytes;
    auto item_end = [&](size_t v) -> size_t {  // virtual bytes of visit slots [0, v)
      if (v == items) return content_bytes;  // (incl. the packed area's tail pad)
      if (packed_first) return v < np ? pl.poff[v] : P + (v - np) * (size_t)SAMPLED_CONTENT_LEN;
      return v <= ns ? v * (size_t)SAMPLED_CONTENT_LEN : pl.sampled_bytes + pl.poff[v - ns];
    };
    auto phys = [&](size_t x) -> size_t { return !packed_first ? x : x < P ? pl.sampled_bytes + x : x - P; };
    auto send = [&](size_t lo, size_t hi, hipStream_t cs) -> hipError_t {  // virtual [lo, hi)
      const size_t cut = packed_first && lo < P && hi > P ? P : hi;
      for (size_t a = lo, b = cut; a < hi; a = b, b = hi) {
        const size_t pa = phys(a);
        const hipError_t e = SD_PATHS_PULL ? pull_host(dev + pa, pin + pa, b - a, cs)
                                           : hipMemcpyAsync(dev + pa, pin + pa, b - a, hipMemcpyHostToDevice, cs);
        if (e != hipSuccess) return e;
      }
      return hipSuccess;
    };
    auto pump = [&]() {
      const size_t meta_hi = staged_h2d_bytes(pl);
      if (hipMemcpyAsync(dev + content_bytes, pin + content_bytes, meta_hi - content_bytes,
                         hipMemcpyHostToDevice, c->copy) != hipSuccess)
        prc = SD_CAS_EHIP;
      size_t ready = 0, sent = 0;
      while (sent < content_bytes) {
        while (ready < items && fin[ready].load(std::memory_order_acquire)) ++ready;
        const size_t hi = item_end(ready);
        // (the first piece goes at STREAM_FIRST bytes: the host link starts sooner; with
        // SD_PATHS_RAMP the piece threshold doubles from there up to STREAM_CHUNK)
        const size_t want = !sent ? STREAM_FIRST
                            : SD_PATHS_RAMP ? std::min(STREAM_CHUNK, STREAM_FIRST << std::min<size_t>(npieces, 16))
                                            : STREAM_CHUNK;
        // (and the whole-file area goes as soon as it is complete, so its hash starts early)
        if (hi > sent && (hi - sent >= want || ready == items ||
                          (packed_first && sent < P && hi >= P))) {
          const auto t0 = std::chrono::steady_clock::now();
          if (first_us < 0 && tr.on) first_us = since(t_pump);
          ++npieces;
          hipStream_t cs = (SD_PATHS_COPY_STREAMS > 1 && (ncopies_all++ & 1)) ? c->copy2 : c->copy;
          if (prc == SD_CAS_OK && send(sent, hi, cs) != hipSuccess) prc = SD_CAS_EHIP;
          if (tr.on) { copy_us += since(t0); last_us = since(t_pump); ++ncopies; }
          sent = hi;
          if (packed_first && !packed_early && sent >= P && prc == SD_CAS_OK) {
            // every whole file has landed: hash them now, on copy2 (idle with one copy
            // stream), so the whole-file and sampled hashes run side by side at the end
            if (SD_PATHS_COPY_STREAMS > 1 &&
                (hipEventRecord(c->copy2_done, c->copy2) != hipSuccess ||
                 hipStreamWaitEvent(c->copy, c->copy2_done, 0) != hipSuccess))
              prc = SD_CAS_EHIP;
            else if (hipEventRecord(c->packed_h2d, c->copy) != hipSuccess ||
                     hipStreamWaitEvent(c->copy2, c->packed_h2d, 0) != hipSuccess)
              prc = SD_CAS_EHIP;
            else if (enqueue_packed(c, pl, pin, dev, c->copy2) != SD_CAS_OK ||
                     hipEventRecord(c->packed_done, c->copy2) != hipSuccess)
              prc = SD_CAS_EHIP;
            packed_early = prc == SD_CAS_OK;
            if (tr.on) tr.note("packed_hash_at", since(t_pump));
          }
        } else if (size_t v; next.load(std::memory_order_relaxed) < items &&
                   (v = next.fetch_add(1)) < items) {
          item(vis(v));  // nothing to copy yet: read a file too (a 16th reader, no extra thread)
          fin[v].store(1, std::memory_order_release);
        } else {
#if defined(__x86_64__)
          __builtin_ia32_pause();
#else
          std::this_thread::yield();
#endif
        }
      }
    };
    c->pool.run2(threads, worker, pump);
    if (SD_PATHS_COPY_STREAMS > 1 && ncopies_all > 1 && prc == SD_CAS_OK) {
      // the copy stream (whose event the hash waits on) also waits for the second one's pieces
      if (hipEventRecord(c->copy2_done, c->copy2) != hipSuccess ||
          hipStreamWaitEvent(c->copy, c->copy2_done, 0) != hipSuccess)
        prc = SD_CAS_EHIP;
    }
    tr.note("copies", (double)ncopies);
    tr.note("copy_api_us", copy_us);
    tr.note("first_copy_at", first_us);
    tr.note("last_copy_at", last_us);
    if (prc) return fail(c, prc, "from_paths: streamed H2D failed");
    return SD_CAS_OK;
  };
  auto finish = [&](size_t w) -> int {
    const int b = (int)(w & 1);
    HIP_TRY(c, hipEventSynchronize(done[b]));
    scatter_keys(plans[w], pin0 + b * slot, out_keys + wstart[w]);
    return SD_CAS_OK;
  };
  for (size_t w = 0; w < nw && rc == 0; w++) {
    const int b = (int)(w & 1);
    if (w >= 2 && (rc = finish(w - 2))) break;  // slot b free again
    const size_t f0 = wstart[w], m = wstart[w + 1] - wstart[w];
    const bool single = nw == 1 && m >= STREAM_MIN_FILES;
    char* pin = pin0 + b * slot;
    char* dev = dev0 + b * slot;
    if (single && SD_PATHS_ZERO_COPY) {
      // A/B (SD_PATHS_ZERO_COPY): no H2D at all — the kernels read the pinned staging
      // straight over the host link and write the keys into it
      if ((rc = gather(w, pin, dev, false))) break;
      tr.mark("gather");
      stage_meta(plans[w], psize.data() + f0, pin);
      rc = enqueue_hash(c, plans[w], m, pin, pin, done[b], 0, 0);
    } else {
      if (single) stage_meta(plans[w], psize.data() + f0, pin);
      if ((rc = gather(w, pin, dev, single))) break;
      tr.mark("gather");
      rc = single ? enqueue_hash(c, plans[w], m, pin, dev, done[b], 0, 0, packed_early)
                  : enqueue_staged(c, plans[w], psize.data() + f0, m, pin, dev, done[b]);
    }
    tr.mark("enqueue");
  }
  for (size_t w = nw >= 2 ? nw - 2 : 0; w < nw && rc == 0; w++) rc = finish(w);
  tr.mark("wait");
  if (rc) (void)hipStreamSynchronize(c->stream);
  if (rc) return rc;
  // whole files whose length is not their metadata size: read them as they are now
  // (fs::read, cas.rs:29) and hash the few of them as one host batch
  std::vector<size_t> ri;
  for (size_t i = 0; i < n; i++)
    if (redo[i] && !status[i]) ri.push_back(i);
  if (!ri.empty()) {
    std::vector<std::vector<uint8_t>> bufs(ri.size());
    std::vector<const uint8_t*> bp;
    std::vector<uint64_t> bl, bs;
    std::vector<size_t> bi;
    for (size_t k = 0; k < ri.size(); k++) {
      const size_t i = ri[k];
      int fd = open(paths[i], O_RDONLY | O_CLOEXEC);
      if (fd < 0) { status[i] = -errno; continue; }
      std::vector<uint8_t>& b = bufs[k];
      struct stat st;
      b.resize(8 + std::max<size_t>(fstat(fd, &st) == 0 ? (size_t)st.st_size : 0, 1 << 16));
      size_t got = 0;
      for (;;) {  // to EOF, whatever fstat said
        if (8 + got == b.size()) b.resize(b.size() * 2);
        ssize_t r = read(fd, b.data() + 8 + got, b.size() - 8 - got);
        if (r < 0) { if (errno == EINTR) continue; status[i] = -errno; break; }
        if (r == 0) break;
        got += (size_t)r;
      }
      close(fd);
      if (status[i]) continue;
      if (got > MAX_PACKED_CONTENT_LEN) {
        // longer than any whole-file message the cas kernels take (the metadata said
        // <= 100 KiB): hash M = le64(size) || content with the validator tree (K3)
        for (int j = 0; j < 8; j++) b[j] = (uint8_t)(sizes[i] >> (8 * j));
        void* d = nullptr;
        uint8_t dg[32];
        int rc2 = hipMalloc(&d, up256(8 + got)) == hipSuccess &&
                          hipMemcpy(d, b.data(), 8 + got, hipMemcpyHostToDevice) == hipSuccess
                      ? sd_cas_checksum_dev(c, d, 8 + got, dg, nullptr)
                      : fail(c, SD_CAS_EHIP, "from_paths: long whole file");
        if (d) (void)hipFree(d);
        if (rc2) return rc2;
        uint64_t key = 0;
        for (int j = 0; j < 8; j++) key = (key << 8) | dg[j];
        out_keys[i] = key;
        continue;
      }
      b.erase(b.begin(), b.begin() + 8);
      b.resize(got);
      bp.push_back(b.data());
      bl.push_back(got);
      bs.push_back(sizes[i]);
      bi.push_back(i);
    }
    if (!bi.empty()) {
      std::vector<uint64_t> k(bi.size());
      rc = sd_cas_generate_cas_ids(c, bp.data(), bl.data(), bs.data(), bi.size(), k.data());
      if (rc) return rc;
      for (size_t j = 0; j < bi.size(); j++) out_keys[bi[j]] = k[j];
    }
  }
  for (size_t i = 0; i < n; i++)
    if (status[i]) out_keys[i] = 0;
  return SD_CAS_OK;
}

// File i's content is at h_content + (i % ring) * stride: ring == n is a plain batch, a
// smaller ring re-sends the same host bytes cyclically (BASELINE config 3's E2E run over
// more files than fit in pinned memory; the H2D volume is the full n files either way).
static int hash_sampled_host_impl(sd_cas_ctx* c, const void* h_content, uint64_t stride,
                                  size_t ring, const uint64_t* h_sizes, size_t n,
                                  uint64_t* h_keys, size_t batch_files) {
  if (!c) return SD_CAS_EINVAL;
  if (n == 0) return SD_CAS_OK;
  if (!h_content || !h_sizes || !h_keys || stride < SAMPLED_CONTENT_LEN || (stride & 15) || !ring)
    return fail(c, SD_CAS_EINVAL, "hash_sampled_host: bad arguments");
  HIP_TRY(c, hipSetDevice(c->device));
  if (batch_files == 0) batch_files = sd_cas_batch_quantum(c);
  batch_files = std::min(batch_files, n);
  // two device slots: [content | sizes | keys], ping-ponged between the copy stream (H2D of
  // batch k+1) and the compute stream (K1 on batch k, then D2H of its keys).  Sizes and keys
  // go through two pinned slots as well: a D2H into pageable caller memory would block this
  // thread until K1 finished and serialise the next H2D behind it.
  const size_t cbytes = up256(batch_files * stride), sbytes = up256(batch_files * 8);
  const size_t slot = cbytes + 2 * sbytes;
  int rc = ensure(c, c->staging, 2 * slot);
  if (rc) return rc;
  if ((rc = ensure_pinned(c, 4 * sbytes))) return rc;
  hipEvent_t ev[4] = {nullptr, nullptr, nullptr, nullptr};  // h2d[0..1], done[0..1]
  int result = SD_CAS_OK;
  for (int i = 0; i < 4 && result == SD_CAS_OK; i++)
    if (hipEventCreateWithFlags(&ev[i], hipEventDisableTiming) != hipSuccess)
      result = fail(c, SD_CAS_EHIP, "hash_sampled_host: event create");
  hipEvent_t* h2d = ev;
  hipEvent_t* done = ev + 2;
  const size_t nb = (n + batch_files - 1) / batch_files;
  auto keys_out = [&](size_t k) -> int {  // batch k's keys: pinned slot -> caller
    const int b = (int)(k & 1);
    const size_t f0 = k * batch_files, m = std::min(batch_files, n - f0);
    if (hipEventSynchronize(done[b]) != hipSuccess)
      return fail(c, SD_CAS_EHIP, "hash_sampled_host: batch %zu", k);
    memcpy(h_keys + f0, (const char*)c->pinned + (2 + b) * sbytes, m * 8);
    return SD_CAS_OK;
  };
  for (size_t k = 0; k < nb && result == SD_CAS_OK; k++) {
    const int b = (int)(k & 1);
    const size_t f0 = k * batch_files, m = std::min(batch_files, n - f0);
    char* base = (char*)c->staging.p + b * slot;
    uint8_t* d_content = (uint8_t*)base;
    uint64_t* d_sizes = (uint64_t*)(base + cbytes);
    uint64_t* d_keys = (uint64_t*)(base + cbytes + sbytes);
    uint64_t* p_sizes = (uint64_t*)((char*)c->pinned + b * sbytes);
    uint64_t* p_keys = (uint64_t*)((char*)c->pinned + (2 + b) * sbytes);
    if (k >= 2 && (result = keys_out(k - 2))) break;  // slot b (device + pinned) free again
    memcpy(p_sizes, h_sizes + f0, m * 8);
    hipError_t e = hipSuccess;
    for (size_t done_f = 0; e == hipSuccess && done_f < m;) {  // <= 2 pieces per ring wrap
      const size_t r0 = (f0 + done_f) % ring, piece = std::min(m - done_f, ring - r0);
      e = hipMemcpyAsync(d_content + done_f * stride, (const char*)h_content + r0 * stride,
                         piece * stride, hipMemcpyHostToDevice, c->copy);
      done_f += piece;
    }
    if (e == hipSuccess) e = hipMemcpyAsync(d_sizes, p_sizes, m * 8, hipMemcpyHostToDevice, c->copy);
    if (e == hipSuccess) e = hipEventRecord(h2d[b], c->copy);
    if (e == hipSuccess) e = hipStreamWaitEvent(c->stream, h2d[b], 0);
    if (e == hipSuccess) e = dispatch_sampled(c, d_content, stride, d_sizes, m, d_keys, c->stream);
    if (e == hipSuccess) e = hipMemcpyAsync(p_keys, d_keys, m * 8, hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipEventRecord(done[b], c->stream);
    if (e != hipSuccess) result = fail(c, SD_CAS_EHIP, "hash_sampled_host: %s", hipGetErrorString(e));
  }
  for (size_t k = nb >= 2 ? nb - 2 : 0; k < nb && result == SD_CAS_OK; k++) result = keys_out(k);
  (void)hipStreamSynchronize(c->stream);
  (void)hipStreamSynchronize(c->copy);
  for (int i = 0; i < 4; i++)
    if (ev[i]) (void)hipEventDestroy(ev[i]);
  return result;
}

int sd_cas_hash_sampled_host(sd_cas_ctx* c, const void* h_content, uint64_t stride,
                             const uint64_t* h_sizes, size_t n, uint64_t* h_keys,
                             size_t batch_files) {
  return hash_sampled_host_impl(c, h_content, stride, n, h_sizes, n, h_keys, batch_files);
}

int sd_cas_hash_sampled_host_ring(sd_cas_ctx* c, const void* h_ring, uint64_t stride,
                                  size_t ring_files, const uint64_t* h_sizes, size_t n,
                                  uint64_t* h_keys, size_t batch_files) {
  return hash_sampled_host_impl(c, h_ring, stride, ring_files, h_sizes, n, h_keys, batch_files);
}

// ---- file_checksum --------------------------------------------------------------------

int sd_cas_checksum_dev(sd_cas_ctx* c, const void* d_data, uint64_t len, uint8_t out[32],
                        void* stream) {
  if (!c || !out) return SD_CAS_EINVAL;
  if ((len && !d_data) || ((uintptr_t)d_data & 15))
    return fail(c, SD_CAS_EINVAL, "checksum: bad data pointer");
  hipStream_t s = pick(c, stream);
  // up to 64 GiB: the batch chain with one buffer (K3b: its wide static grid and spread
  // block level ran 2.99 vs K3's 2.88 TB/s on the same 16 GiB, profiles/r02b_validator_batch.log)
  constexpr uint64_t BATCH_MAX = 64ull << 30;
  const bool batch = len <= BATCH_MAX;
  int rc = ensure(c, c->ws, batch ? checksum_batch_workspace_bytes(1, len) : checksum_workspace_bytes(len));
  if (rc) return rc;
  uint32_t* d_out = (uint32_t*)c->d_scalar;  // d_scalar[0..3]: digest; [4], [5]: offs, lens
  HIP_TRY(c, sd_ws_acquire(c, s));
  if (batch) {
    uint64_t* d_ol = c->d_scalar + 4;
    HIP_TRY(c, checksum_single_setup(d_ol, len, (uint32_t*)(c->d_scalar + 6), s));
    HIP_TRY(c, checksum_batch_device((const uint8_t*)d_data, len, d_ol, d_ol + 1, 1, d_out,
                                     (uint32_t*)(c->d_scalar + 6), c->ws.p, s));
  } else {
    HIP_TRY(c, checksum_device((const uint8_t*)d_data, len, 0, true, d_out, c->ws.p, s));
  }
  HIP_TRY(c, hipMemcpyAsync(out, d_out, 32, hipMemcpyDeviceToHost, s));
  HIP_TRY(c, sd_ws_release(c, s));
  HIP_TRY(c, hipStreamSynchronize(s));
  return SD_CAS_OK;
}

// file_checksum(path) (validation/hash.rs:11-25): the reference issues one read() of
// BLOCK_LEN = 1 MiB per iteration into one hasher and stops at the FIRST read that returns
// fewer bytes — the end of a regular file on a local filesystem, but after the first short
// read on anything that returns short reads before its end (procfs seq_files give about one
// page per read, FIFOs and FUSE/network mounts whatever is ready).
// Two read modes, one result:
//   * parallel (regular files): the file streams through two pinned segment buffers of up
//     to 64 MiB (a segment = one complete 65,536-chunk subtree, hashed on the GPU while the
//     pool reads the next one with pread pieces) until a segment comes back short; st_size
//     only sizes the buffers (a file that outgrows its first buffer is re-read with full-size
//     segments).  A regular file whose reads show it is not read like a local file — a short
//     pread followed by more data, or an end before st_size — is redone sequentially;
//   * sequential (everything else, and those redos): hash.rs's loop literally, 1 MiB read()s
//     from the start, stopping after the first short one, into the same segment pipeline.
// The segment CVs are merged on the GPU (pair-and-promote, ROOT on the last parent); a file
// of one segment is hashed with ROOT inside the segment.
static int cv_capacity(sd_cas_ctx* c, DevBuf& cvb, size_t need_cvs, hipStream_t s) {
  if (need_cvs * 32 <= cvb.bytes) return SD_CAS_OK;
  DevBuf nb;
  const size_t want = std::max<size_t>(need_cvs * 2 * 32, 1 << 16);
  HIP_TRY(c, hipStreamSynchronize(s));
  if (hipMalloc(&nb.p, want) != hipSuccess) {
    (void)hipGetLastError();
    return fail(c, SD_CAS_ENOMEM, "hipMalloc(%zu) failed", want);
  }
  nb.bytes = want;
  if (cvb.p) {
    HIP_TRY(c, hipMemcpy(nb.p, cvb.p, cvb.bytes, hipMemcpyDeviceToDevice));
    HIP_TRY(c, hipFree(cvb.p));
  }
  cvb = nb;
  return SD_CAS_OK;
}

int sd_cas_file_checksum(sd_cas_ctx* c, const char* path, char out_hex[65], int* err_no) {
  if (!c || !path || !out_hex) return SD_CAS_EINVAL;
  if (err_no) *err_no = 0;
  HIP_TRY(c, hipSetDevice(c->device));
  int fd = open(path, O_RDONLY | O_CLOEXEC);
  if (fd < 0) {
    if (err_no) *err_no = errno;
    return fail(c, SD_CAS_EIO, "open(%s): %s", path, strerror(errno));
  }
  struct stat st;
  if (fstat(fd, &st) != 0) {
    if (err_no) *err_no = errno;
    close(fd);
    return fail(c, SD_CAS_EIO, "fstat(%s): %s", path, strerror(errno));
  }
  const uint64_t SEG = 64ull << 20;  // 65,536 chunks: a complete left subtree
  constexpr uint64_t PIECE = 4ull << 20;  // pool read unit (one reader tops out near 5-10 GB/s)
  constexpr uint64_t BLOCK_LEN = 1ull << 20;  // hash.rs:9
  static_assert((64ull << 20) % BLOCK_LEN == 0, "a segment holds whole hash.rs reads");
  bool seq = !S_ISREG(st.st_mode);
  // segment capacity: the whole file plus room to see EOF, capped at one subtree (the
  // sequential mode reads whole 1 MiB blocks: full segments)
  uint64_t cap = seq ? SEG : std::min<uint64_t>(SEG, (((uint64_t)st.st_size + 1 + 4095) / 4096) * 4096);
  hipStream_t s = c->stream;
  int rc = SD_CAS_OK;
  hipEvent_t done[2] = {nullptr, nullptr};
  for (int i = 0; i < 2; i++)
    if (hipEventCreateWithFlags(&done[i], hipEventDisableTiming) != hipSuccess) {
      close(fd);
      for (int k = 0; k < i; k++) (void)hipEventDestroy(done[k]);
      return fail(c, SD_CAS_EHIP, "file_checksum: event create");
    }
  bool irregular = false;  // parallel mode saw reads that a local regular file never gives
  bool seq_stopped = false;  // sequential mode: the first short read has happened
  // parallel: read segment `sgi` into dst with pread pieces; its length (< cap at EOF) or -errno
  auto read_seg_par = [&](uint64_t sgi, char* dst) -> int64_t {
    const uint64_t off = sgi * cap;
    const uint64_t npieces = (cap + PIECE - 1) / PIECE;
    std::atomic<uint64_t> next{0}, eof{cap}, data_end{0};
    std::atomic<int> rd_err{0};
    std::atomic<bool> short_then_more{false};
    c->pool.run((unsigned)std::min<uint64_t>(8, npieces), [&]() {
      for (uint64_t p; (p = next.fetch_add(1)) < npieces && !rd_err.load();) {
        const uint64_t p0 = p * PIECE, pn = std::min(PIECE, cap - p0);
        if (p0 >= eof.load()) break;
        uint64_t got = 0;
        bool was_short = false;
        while (got < pn) {
          ssize_t r = pread(fd, dst + p0 + got, pn - got, (off_t)(off + p0 + got));
          if (r < 0 && errno == EINTR) continue;
          if (r < 0) { rd_err.store(errno); break; }
          if (r == 0) break;
          if (was_short) short_then_more.store(true);  // data after a short read
          if ((uint64_t)r < pn - got) was_short = true;
          got += (uint64_t)r;
        }
        if (got) {
          uint64_t cur = data_end.load();
          while (p0 + got > cur && !data_end.compare_exchange_weak(cur, p0 + got)) {}
        }
        if (got < pn) {  // eof = min(eof, p0 + got)
          uint64_t cur = eof.load();
          while (p0 + got < cur && !eof.compare_exchange_weak(cur, p0 + got)) {}
        }
      }
    });
    if (int e = rd_err.load()) return -(int64_t)e;
    // bytes past the first end (a short piece whose successor still had data)
    if (short_then_more.load() || data_end.load() > eof.load()) irregular = true;
    return (int64_t)eof.load();
  };
  // sequential: hash.rs:15-21 — 1 MiB read()s in order, stop after the first short one
  auto read_seg_seq = [&](char* dst) -> int64_t {
    if (seq_stopped) return 0;
    uint64_t got = 0;
    while (got < cap) {
      ssize_t r = read(fd, dst + got, BLOCK_LEN);
      if (r < 0 && errno == EINTR) continue;
      if (r < 0) return -(int64_t)errno;
      got += (uint64_t)r;
      if ((uint64_t)r != BLOCK_LEN) { seq_stopped = true; break; }
    }
    return (int64_t)got;
  };
  auto read_seg = [&](uint64_t sgi, char* dst) -> int64_t {
    return seq ? read_seg_seq(dst) : read_seg_par(sgi, dst);
  };
  uint8_t digest[32];
  for (int attempt = 0; attempt < 3; attempt++) {
    const size_t sb = up256(cap + 16);
    if ((rc = ensure_pinned(c, 2 * sb)) || (rc = ensure(c, c->staging, 2 * sb))) break;
    if ((rc = ensure(c, c->ws, std::max(checksum_workspace_bytes(cap), checksum_workspace_bytes(1 << 20)))))
      break;
    char* pin[2] = {(char*)c->pinned, (char*)c->pinned + sb};
    char* dev[2] = {(char*)c->staging.p, (char*)c->staging.p + sb};
    if (hipError_t e = sd_ws_acquire(c, s); e != hipSuccess) {
      rc = fail(c, SD_CAS_EHIP, "file_checksum: %s", hipGetErrorString(e));
      break;
    }
    // segment k is dispatched once it is known whether it is the only one (k == 0 waits for
    // segment 1's read); ROOT sits inside it only then
    auto dispatch = [&](uint64_t sgi, uint64_t len, bool only) -> int {
      const int b = (int)(sgi & 1);
      int r2 = cv_capacity(c, c->cvbuf, sgi + 1, s);
      if (r2) return r2;
      hipError_t e = hipMemcpyAsync(dev[b], pin[b], up16(len), hipMemcpyHostToDevice, s);
      if (e == hipSuccess)
        e = checksum_device((const uint8_t*)dev[b], len, (sgi * cap) >> 10, only,
                            (uint32_t*)c->cvbuf.p + 8 * sgi, c->ws.p, s);
      if (e == hipSuccess) e = hipEventRecord(done[b], s);
      if (e != hipSuccess) return fail(c, SD_CAS_EHIP, "checksum segment: %s", hipGetErrorString(e));
      return SD_CAS_OK;
    };
    auto io_fail = [&](int64_t neg) {
      if (err_no) *err_no = (int)-neg;
      return fail(c, SD_CAS_EIO, "read(%s): %s", path, strerror((int)-neg));
    };
    enum { DONE, GROW, GO_SEQ } next = DONE;
    uint64_t nseg = 1, total = 0;
    int64_t len0 = read_seg(0, pin[0]);
    if (len0 < 0) {
      rc = io_fail(len0);
    } else if (irregular) {
      next = GO_SEQ;
    } else if ((uint64_t)len0 == cap && cap < SEG) {
      next = GROW;  // grew past the buffer
    } else if ((uint64_t)len0 < cap) {
      total = (uint64_t)len0;
      rc = dispatch(0, (uint64_t)len0, true);
    } else {  // a full first segment: more may follow
      total = (uint64_t)len0;
      for (uint64_t sgi = 1;; sgi++) {
        const int b = (int)(sgi & 1);
        if (sgi >= 2 && hipEventSynchronize(done[b]) != hipSuccess) { rc = fail(c, SD_CAS_EHIP, "checksum: segment sync"); break; }
        const int64_t ln = read_seg(sgi, pin[b]);
        if (ln < 0) { rc = io_fail(ln); break; }
        if (irregular) { next = GO_SEQ; break; }
        total += (uint64_t)ln;
        if (sgi == 1) {  // segment 0 is the only one iff nothing follows it
          if ((rc = dispatch(0, (uint64_t)len0, ln == 0))) break;
        }
        if (ln == 0) { nseg = sgi; break; }
        if ((rc = dispatch(sgi, (uint64_t)ln, false))) break;
        if ((uint64_t)ln < cap) { nseg = sgi + 1; break; }
      }
    }
    // a regular file that ended before its st_size (it shrank, or a read came back short at
    // a piece boundary): redo it the way hash.rs reads
    if (rc == SD_CAS_OK && next == DONE && !seq && total < (uint64_t)st.st_size) next = GO_SEQ;
    if (rc == SD_CAS_OK && next == DONE) {
      uint32_t* d_out = (uint32_t*)c->d_scalar;
      hipError_t e = hipSuccess;
      // reduce_cvs_device ping-pongs ceil(nseg / 256) CVs per level through ws
      const size_t red_ws = 2 * up256((nseg + 255) / 256 * 32) + 512;
      if (nseg > 1) rc = ensure(c, c->ws, red_ws);
      if (rc == SD_CAS_OK) {
        if (nseg == 1) e = hipMemcpyAsync(d_out, c->cvbuf.p, 32, hipMemcpyDeviceToDevice, s);
        else e = reduce_cvs_device((uint32_t*)c->cvbuf.p, nseg, d_out, c->ws.p, s);
        if (e == hipSuccess) e = hipMemcpyAsync(digest, d_out, 32, hipMemcpyDeviceToHost, s);
        if (e == hipSuccess) e = hipStreamSynchronize(s);
        if (e != hipSuccess) rc = fail(c, SD_CAS_EHIP, "checksum reduce: %s", hipGetErrorString(e));
      }
    }
    (void)hipStreamSynchronize(s);  // no segment copy may still read the pinned buffers
    (void)sd_ws_release(c, s);
    if (rc != SD_CAS_OK || next == DONE) break;
    if (next == GROW) {
      cap = SEG;
    } else {  // GO_SEQ: from the start, hash.rs's reads
      seq = true;
      cap = SEG;
      irregular = false;
      if (lseek(fd, 0, SEEK_SET) != 0) {
        if (err_no) *err_no = errno;
        rc = fail(c, SD_CAS_EIO, "lseek(%s): %s", path, strerror(errno));
        break;
      }
    }
    if (attempt == 2) rc = fail(c, SD_CAS_EIO, "file_checksum(%s): no stable read", path);
  }
  close(fd);
  (void)hipStreamSynchronize(s);
  (void)hipEventDestroy(done[0]);
  (void)hipEventDestroy(done[1]);
  if (rc) return rc;
  static const char* hx = "0123456789abcdef";
  for (int i = 0; i < 32; i++) { out_hex[2 * i] = hx[digest[i] >> 4]; out_hex[2 * i + 1] = hx[digest[i] & 15]; }
  out_hex[64] = 0;
  return SD_CAS_OK;
}

// ---- the validator job over many files -----------------------------------------------

int sd_cas_checksums_dev(sd_cas_ctx* c, const void* d_arena, uint64_t arena_bytes,
                         const uint64_t* d_offs, const uint64_t* d_lens, size_t n, uint8_t* d_out,
                         void* stream) {
  if (!c) return SD_CAS_EINVAL;
  if (n == 0) return SD_CAS_OK;
  if (!d_arena || !d_offs || !d_lens || !d_out || ((uintptr_t)d_arena & 15) ||
      ((uintptr_t)d_out & 3) || n > (1u << 24))
    return fail(c, SD_CAS_EINVAL, "checksums: bad arguments");
  HIP_TRY(c, hipSetDevice(c->device));
  hipStream_t s = pick(c, stream);
  int rc = ensure(c, c->ws, checksum_batch_workspace_bytes(n, arena_bytes));
  if (rc) return rc;
  uint32_t* d_bad = (uint32_t*)(c->d_scalar + 6);
  uint32_t bad = 0;
  HIP_TRY(c, sd_ws_acquire(c, s));
  HIP_TRY(c, hipMemsetAsync(d_bad, 0, 4, s));
  HIP_TRY(c, checksum_batch_device((const uint8_t*)d_arena, arena_bytes, d_offs, d_lens, n,
                                   (uint32_t*)d_out, d_bad, c->ws.p, s));
  HIP_TRY(c, hipMemcpyAsync(&bad, d_bad, 4, hipMemcpyDeviceToHost, s));
  HIP_TRY(c, sd_ws_release(c, s));
  HIP_TRY(c, hipStreamSynchronize(s));
  if (bad)
    return fail(c, SD_CAS_EINVAL, "checksums: %s",
                (bad & 1) ? "a buffer is longer than 64 GiB"
                          : (bad & 4) ? "a buffer is misaligned or extends past arena_bytes"
                                      : "the buffers' subtrees exceed arena_bytes' bound (overlapping buffers?)");
  return SD_CAS_OK;
}

// file_checksum over many paths.  Windows of up to CK_WIN bytes / CK_WIN_FILES files in
// index order, double-buffered: the pool reads window w (one slot of up128(st_size + 1) per
// file: the spare byte shows EOF, so a file that grew since stat fills its slot and is
// redone by the streaming path) into one pinned slot while the GPU copies and hashes window
// w-1 from the other.  Pinned slot layout: offs | lens | digests | data.
int sd_cas_file_checksums(sd_cas_ctx* c, const char* const* paths, size_t n, char* out_hex,
                          int32_t* status) {
  if (!c) return SD_CAS_EINVAL;
  if (n == 0) return SD_CAS_OK;
  if (!paths || !out_hex || !status) return fail(c, SD_CAS_EINVAL, "file_checksums: null argument");
  HIP_TRY(c, hipSetDevice(c->device));
  constexpr uint64_t CK_WIN = 128ull << 20;  // data bytes per window
  constexpr uint64_t CK_BIG = CK_WIN / 2;    // larger files stream on their own (64 MiB segments)
  constexpr size_t CK_WIN_FILES = 32768;
  constexpr size_t HDR = CK_WIN_FILES * (8 + 8 + 32);
  constexpr size_t SLOT = HDR + CK_WIN + 256;
  enum : uint8_t { K_BATCH = 0, K_STREAM = 1, K_ERROR = 2 };
  std::vector<uint64_t> fsize(n, 0);
  std::vector<uint8_t> kind(n, K_BATCH);
  for (size_t i = 0; i < n; i++) { status[i] = 0; out_hex[65 * i] = 0; }
  {  // stat pass
    std::atomic<size_t> next{0};
    c->pool.run(std::max(1u, std::min(16u, (unsigned)((n + 63) / 64))), [&]() {
      for (size_t i; (i = next.fetch_add(1)) < n;) {
        struct stat st;
        if (stat(paths[i], &st) != 0) { status[i] = -errno; kind[i] = K_ERROR; continue; }
        fsize[i] = (uint64_t)st.st_size;
        // not a regular file (FIFO, device, ...): hash.rs's sequential reads, streamed
        if (fsize[i] > CK_BIG || !S_ISREG(st.st_mode)) kind[i] = K_STREAM;
      }
    });
  }
  // windows: [w0, w1) file ranges in index order
  std::vector<size_t> wstart{0};
  {
    uint64_t bytes = 0;
    size_t files = 0;
    for (size_t i = 0; i < n; i++) {
      if (kind[i] != K_BATCH) continue;
      const uint64_t need = up128(fsize[i] + 1);
      if (files && (bytes + need > CK_WIN || files == CK_WIN_FILES)) {
        wstart.push_back(i);
        bytes = 0;
        files = 0;
      }
      bytes += need;
      files++;
    }
    wstart.push_back(n);
  }
  const size_t nw = wstart.size() - 1;
  int rc = ensure_pinned(c, 2 * SLOT);
  if (rc) return rc;
  if ((rc = ensure(c, c->staging, 2 * SLOT))) return rc;
  if ((rc = ensure(c, c->ws, checksum_batch_workspace_bytes(CK_WIN_FILES, CK_WIN)))) return rc;
  hipStream_t s = c->stream;
  hipEvent_t done[2] = {nullptr, nullptr};
  for (int b = 0; b < 2; b++)
    if (hipEventCreateWithFlags(&done[b], hipEventDisableTiming) != hipSuccess) {
      if (done[0]) (void)hipEventDestroy(done[0]);
      return fail(c, SD_CAS_EHIP, "file_checksums: event create");
    }
  std::vector<size_t> members[2];  // file index of each batch entry of the window in a slot
  static const char* hx = "0123456789abcdef";
  auto emit = [&](int b) {  // the window in slot b is complete: digests -> hex
    const uint8_t* dg = (const uint8_t*)c->pinned + (size_t)b * SLOT + CK_WIN_FILES * 16;
    for (size_t k = 0; k < members[b].size(); k++) {
      char* o = out_hex + 65 * members[b][k];
      for (int j = 0; j < 32; j++) { o[2 * j] = hx[dg[32 * k + j] >> 4]; o[2 * j + 1] = hx[dg[32 * k + j] & 15]; }
      o[64] = 0;
    }
    members[b].clear();
  };
  bool pending[2] = {false, false};
  uint32_t* d_bad = (uint32_t*)(c->d_scalar + 6);
  {
    hipError_t e = sd_ws_acquire(c, s);
    if (e == hipSuccess) e = hipMemsetAsync(d_bad, 0, 4, s);
    if (e != hipSuccess) rc = fail(c, SD_CAS_EHIP, "file_checksums: %s", hipGetErrorString(e));
  }
  for (size_t w = 0; w < nw && rc == SD_CAS_OK; w++) {
    const int b = (int)(w & 1);
    if (pending[b]) {  // slot b's previous window: copied, hashed and its digests back
      if (hipEventSynchronize(done[b]) != hipSuccess) { rc = fail(c, SD_CAS_EHIP, "file_checksums: sync"); break; }
      emit(b);
      pending[b] = false;
    }
    char* pin = (char*)c->pinned + (size_t)b * SLOT;
    uint64_t* h_offs = (uint64_t*)pin;
    uint64_t* h_lens = h_offs + CK_WIN_FILES;
    char* data = pin + HDR;
    std::vector<size_t>& mem = members[b];
    std::vector<uint64_t> cap;
    uint64_t o = 0;
    for (size_t i = wstart[w]; i < wstart[w + 1]; i++) {
      if (kind[i] != K_BATCH) continue;
      h_offs[mem.size()] = o;
      cap.push_back(up128(fsize[i] + 1));
      o += cap.back();
      mem.push_back(i);
    }
    const size_t m = mem.size();
    if (m == 0) continue;
    std::atomic<size_t> next{0};
    c->pool.run(std::max(1u, std::min(16u, (unsigned)((m + 3) / 4))), [&]() {
      for (size_t k; (k = next.fetch_add(1)) < m;) {
        const size_t i = mem[k];
        int fd = open(paths[i], O_RDONLY | O_CLOEXEC);
        if (fd < 0) { status[i] = -errno; kind[i] = K_ERROR; h_lens[k] = 0; continue; }
        uint64_t got = 0;
        bool was_short = false, irregular = false;
        while (got < cap[k]) {
          ssize_t r = pread(fd, data + h_offs[k] + got, cap[k] - got, (off_t)got);
          if (r < 0 && errno == EINTR) continue;
          if (r < 0) { status[i] = -errno; kind[i] = K_ERROR; break; }
          if (r == 0) break;  // EOF
          if (was_short) irregular = true;  // data after a short read: not a local file
          if ((uint64_t)r < cap[k] - got) was_short = true;
          got += (uint64_t)r;
        }
        close(fd);
        // grew past its slot, or read unlike a local regular file (a short read before the
        // end, or an end before st_size): sd_cas_file_checksum afterwards, which reads such
        // a file exactly as hash.rs:15-21 does (1 MiB reads, stop at the first short one)
        if (kind[i] == K_BATCH && (got == cap[k] || irregular || got < fsize[i])) kind[i] = K_STREAM;
        h_lens[k] = kind[i] == K_BATCH ? got : 0;
      }
    });
    // entries that failed or grew are hashed as empty buffers and ignored
    hipError_t e = hipMemcpyAsync((char*)c->staging.p + (size_t)b * SLOT, pin, CK_WIN_FILES * 16,
                                  hipMemcpyHostToDevice, s);
    if (e == hipSuccess)
      e = hipMemcpyAsync((char*)c->staging.p + (size_t)b * SLOT + HDR, data, o, hipMemcpyHostToDevice, s);
    char* dbase = (char*)c->staging.p + (size_t)b * SLOT;
    if (e == hipSuccess)
      e = checksum_batch_device((const uint8_t*)(dbase + HDR), o, (const uint64_t*)dbase,
                                (const uint64_t*)dbase + CK_WIN_FILES, m,
                                (uint32_t*)(dbase + CK_WIN_FILES * 16), d_bad, c->ws.p, s);
    if (e == hipSuccess)
      e = hipMemcpyAsync(pin + CK_WIN_FILES * 16, dbase + CK_WIN_FILES * 16, m * 32,
                         hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipEventRecord(done[b], s);
    if (e != hipSuccess) { rc = fail(c, SD_CAS_EHIP, "file_checksums window: %s", hipGetErrorString(e)); break; }
    pending[b] = true;
  }
  uint32_t bad = 0;
  if (rc == SD_CAS_OK) {
    hipError_t e = hipMemcpyAsync(&bad, d_bad, 4, hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (e != hipSuccess) rc = fail(c, SD_CAS_EHIP, "file_checksums: %s", hipGetErrorString(e));
    else if (bad) rc = fail(c, SD_CAS_EHIP, "file_checksums: batch work list overflow");
  }
  (void)sd_ws_release(c, s);
  (void)hipStreamSynchronize(s);
  for (int b = 0; b < 2; b++) {
    if (rc == SD_CAS_OK && pending[b]) emit(b);
    (void)hipEventDestroy(done[b]);
  }
  if (rc) return rc;
  // big files and files that grew: the streaming path, one at a time (after the windows:
  // it reuses the pinned and device staging)
  for (size_t i = 0; i < n; i++) {
    if (kind[i] != K_STREAM) continue;
    char* o = out_hex + 65 * i;
    int err_no = 0;
    const int r = sd_cas_file_checksum(c, paths[i], o, &err_no);
    if (r == SD_CAS_EIO) { status[i] = -(err_no ? err_no : EIO); o[0] = 0; continue; }
    if (r) return r;
  }
  for (size_t i = 0; i < n; i++)
    if (status[i]) out_hex[65 * i] = 0;
  return SD_CAS_OK;
}

// ---- synthetic inputs ----------------------------------------------------------------

int sd_cas_synth_sampled_dev(sd_cas_ctx* c, uint64_t seed, uint64_t file0, size_t n,
                             uint32_t dup_permille, void* d_content, uint64_t stride,
                             uint64_t* d_sizes, void* stream) {
  if (!c) return SD_CAS_EINVAL;
  if (n == 0) return SD_CAS_OK;
  if (!d_content || !d_sizes || stride < SAMPLED_CONTENT_LEN || (stride & 15) || dup_permille > 1000)
    return fail(c, SD_CAS_EINVAL, "synth_sampled: bad arguments");
  HIP_TRY(c, synth_sampled(seed, file0, n, dup_permille, (uint8_t*)d_content, stride, d_sizes,
                           pick(c, stream)));
  return SD_CAS_OK;
}

int sd_cas_synth_small_dev(sd_cas_ctx* c, uint64_t seed, uint64_t file0, size_t n,
                           uint32_t dup_permille, uint64_t* d_sizes, uint32_t* d_lens,
                           uint64_t* d_offs, void* d_arena, uint64_t* out_arena_bytes,
                           void* stream) {
  if (!c) return SD_CAS_EINVAL;
  if (!d_sizes || !d_lens || !d_offs || dup_permille > 1000)
    return fail(c, SD_CAS_EINVAL, "synth_small: bad arguments");
  hipStream_t s = pick(c, stream);
  if (n == 0) { if (out_arena_bytes) *out_arena_bytes = 16; return SD_CAS_OK; }
  HIP_TRY(c, synth_small_sizes(seed, file0, n, dup_permille, d_sizes, d_lens, s));
  // offsets: 128-B aligned packing (see up128), computed on the host from the lens
  std::vector<uint32_t> lens(n);
  HIP_TRY(c, hipMemcpyAsync(lens.data(), d_lens, n * 4, hipMemcpyDeviceToHost, s));
  HIP_TRY(c, hipStreamSynchronize(s));
  std::vector<uint64_t> offs(n);
  uint64_t o = 0;
  for (size_t i = 0; i < n; i++) { offs[i] = o; o += up128(lens[i]); }
  o += 16;
  if (out_arena_bytes) *out_arena_bytes = o;
  HIP_TRY(c, hipMemcpyAsync(d_offs, offs.data(), n * 8, hipMemcpyHostToDevice, s));
  if (d_arena) HIP_TRY(c, synth_small_content(seed, file0, n, dup_permille, d_offs, d_lens,
                                              (uint8_t*)d_arena, s));
  HIP_TRY(c, hipStreamSynchronize(s));
  return SD_CAS_OK;
}

int sd_cas_synth_small_content_dev(sd_cas_ctx* c, uint64_t seed, uint64_t file0, size_t n,
                                   uint32_t dup_permille, const uint64_t* d_offs,
                                   const uint32_t* d_lens, void* d_arena, void* stream) {
  if (!c) return SD_CAS_EINVAL;
  if (!d_offs || !d_lens || !d_arena || dup_permille > 1000 || ((uintptr_t)d_arena & 15))
    return fail(c, SD_CAS_EINVAL, "synth_small_content: bad arguments");
  if (n == 0) return SD_CAS_OK;
  HIP_TRY(c, synth_small_content(seed, file0, n, dup_permille, d_offs, d_lens,
                                 (uint8_t*)d_arena, pick(c, stream)));
  return SD_CAS_OK;
}

int sd_cas_synth_stream_dev(sd_cas_ctx* c, uint64_t seed, uint64_t file, uint64_t byte_off,
                            uint64_t len, void* d_out, void* stream) {
  if (!c) return SD_CAS_EINVAL;
  if (len && (!d_out || (byte_off & 7) || ((uintptr_t)d_out & 7)))
    return fail(c, SD_CAS_EINVAL, "synth_stream: bad arguments");
  HIP_TRY(c, synth_stream(seed, file, byte_off, len, (uint8_t*)d_out, pick(c, stream)));
  return SD_CAS_OK;
}

int sd_cas_synth_roots_dev(sd_cas_ctx* c, uint64_t seed, uint64_t file0, size_t n,
                           uint32_t dup_permille, uint64_t* d_roots, void* stream) {
  if (!c) return SD_CAS_EINVAL;
  if (n && !d_roots) return fail(c, SD_CAS_EINVAL, "synth_roots: null");
  HIP_TRY(c, synth_roots(seed, file0, n, dup_permille, d_roots, pick(c, stream)));
  return SD_CAS_OK;
}

}  // extern "C"
