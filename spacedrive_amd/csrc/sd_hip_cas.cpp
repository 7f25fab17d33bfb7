// sd_hip_cas.cpp — the C ABI (include/sd_hip_cas.h) over the gfx950 kernels: contexts,
// device-resident cas, grouping, the fused chain, link emission, synthetic inputs (the
// host-buffer/path entry points are in host_paths.cpp, the validator's in validator_host.cpp).
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
#include <ctype.h>
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
uint32_t sd_dbg_violations_links();
}  // namespace sdcas
// debug library only (libsd_hip_cas_debug.so, not in the ABI header): invariant violations
// counted by the device checks of sd_debug.h since the library was loaded
extern "C" uint64_t sd_cas_debug_violations(void) {
  return (uint64_t)sd_dbg_violations_group_hash() + sd_dbg_violations_group() +
         sd_dbg_violations_checksum() + sd_dbg_violations_links();
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

// The gather pool's CPUs: the GPU's NUMA node (its PCI device's sysfs numa_node and the node's
// cpulist), intersected with the CPUs this process may use.  On a two-socket host a reader on
// the far socket copies page-cache bytes across the socket link into staging that the DMA then
// reads back across it again; round 6 measured the file path bimodal between processes (~52 vs
// ~40 GB/s, profiles/r06/validator/) before binding.  SD_CAS_POOL_NUMA=0 leaves the pool
// unbound (A/B); nothing is bound when the node or its CPUs cannot be read.
static void bind_pool_to_gpu_node(sd_cas_ctx* c) {
  const char* e = getenv("SD_CAS_POOL_NUMA");
  char bus[64] = {0};
  if (hipDeviceGetPCIBusId(bus, sizeof bus, c->device) != hipSuccess) return;
  for (char* q = bus; *q; ++q) *q = (char)tolower((unsigned char)*q);
  char path[160];
  snprintf(path, sizeof path, "/sys/bus/pci/devices/%s/numa_node", bus);
  FILE* f = fopen(path, "r");
  int node = -1;
  if (f) {
    if (fscanf(f, "%d", &node) != 1) node = -1;
    fclose(f);
  }
  c->numa_node = node;
  if (node < 0 || (e && strcmp(e, "0") == 0)) return;
  snprintf(path, sizeof path, "/sys/devices/system/node/node%d/cpulist", node);
  f = fopen(path, "r");
  if (!f) return;
  char list[4096] = {0};
  const bool got = fgets(list, sizeof list, f) != nullptr;
  fclose(f);
  if (!got) return;
  cpu_set_t allowed, cpus;
  CPU_ZERO(&cpus);
  if (sched_getaffinity(0, sizeof allowed, &allowed) != 0) return;
  int n = 0;
  for (char* q = list; *q && *q != '\n';) {  // "0-63,128-191"
    char* end;
    long a = strtol(q, &end, 10), b = a;
    if (end == q) break;
    if (*end == '-') b = strtol(end + 1, &end, 10);
    for (long cpu = a; cpu <= b && cpu < CPU_SETSIZE; ++cpu)
      if (CPU_ISSET(cpu, &allowed)) { CPU_SET(cpu, &cpus); ++n; }
    q = *end == ',' ? end + 1 : end;
  }
  // bind only where the node offers the pool's 16 threads a CPU each (a process confined to a
  // few of the node's CPUs keeps its own placement)
  if (n >= 16) c->pool.set_cpus(cpus, n);
}

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
    // test knob: a lower distinct-key bound for the fused chain's region tables, so that the
    // tables' overflow paths (a region's own global table, and a full region's regroup from
    // the whole key array) run on K1G output — uniform BLAKE3 keys never reach the real bound
    const char* f = getenv("SD_CAS_TEST_TABLE_FILL");
    c->test_table_fill = f && *f ? (uint32_t)strtoul(f, nullptr, 10) : 0u;
    //  results stay exact with it set, but every fused grouping then takes the
    // slow overflow paths: never silent
    if (c->test_table_fill)
      fprintf(stderr, "sd_hip_cas: SD_CAS_TEST_TABLE_FILL=%u (test knob): the fused grouping's "
              "region tables overflow at %u distinct keys (exact, much slower)\n",
              c->test_table_fill, c->test_table_fill);
  }
  bind_pool_to_gpu_node(c);
  // the pool's readers on private descriptor tables (HostPool::set_private_fds)
  const char* pf = getenv("SD_CAS_POOL_PRIVATE_FDS");
  const bool private_fds = !(pf && pf[0] == '0');
  c->pool.set_private_fds(private_fds);
  if (c->trace)
    fprintf(stderr, "sd_cas_trace ctx device=%d numa_node=%d pool_cpus=%d private_fds=%d\n", device,
            c->numa_node, c->pool.bound_cpus(), (int)private_fds);
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
hipError_t sd_dispatch_sampled(sd_cas_ctx* c, const uint8_t* content, uint64_t stride,
                               const uint64_t* sizes, size_t n, uint64_t* keys, hipStream_t s) {
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
  HIP_TRY(c, sd_dispatch_sampled(c, (const uint8_t*)d_content, stride, d_sizes, n, d_keys,
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
                                  c->region_keys[k], n, skeys, sfile, c->test_table_fill, s);
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

int sd_cas_identifier_links_ex_dev(sd_cas_ctx* c, const uint64_t* d_keys, const uint8_t* d_state,
                                   size_t n, uint32_t chunk, const uint64_t* d_seed_keys,
                                   const uint32_t* d_seed_objects, size_t n_seed,
                                   const uint32_t* d_pre_objects, uint32_t* d_step,
                                   uint32_t* d_object, uint8_t* d_action, uint64_t* h_step_counts,
                                   size_t max_steps, uint64_t* out_steps, void* stream) {
  if (!c) return SD_CAS_EINVAL;
  const size_t steps_total = sd_cas_identifier_max_steps(n, chunk);
  if (chunk == 0 || n >= (1ull << 32) || !out_steps || max_steps < steps_total ||
      (n && (!d_keys || !d_step || !d_object || !d_action || !h_step_counts)) ||
      (n_seed && (!d_seed_keys || !d_seed_objects)))
    return fail(c, SD_CAS_EINVAL, "identifier_links: bad arguments");
  // a seeded grouping tags rows with LINKS_ROW_FLAG: rows and Object ids below 2^31 (rows
  // that already own an Object run the seeded grouping too)
  const bool seeded = n_seed > 0 || d_pre_objects;
  if (seeded && (n >= LINKS_ROW_FLAG || n_seed >= LINKS_ROW_FLAG || n + n_seed >= (1ull << 32)))
    return fail(c, SD_CAS_EINVAL, "identifier_links: %zu rows + %zu existing Objects exceed 2^31",
                n, n_seed);
  *out_steps = 0;
  for (size_t k = 0; k < 2 * steps_total; k++) h_step_counts[k] = 0;
  if (n == 0) return SD_CAS_OK;
  hipStream_t s = pick(c, stream);
  // staging (this call is blocking): rep | hkeys | hrows | minrow | orphans | starts | counts |
  // [event block offsets | scan tiles | key filter] | 4 counters; the seeded grouping runs over
  // the hashed rows + the existing Objects' keys.  Rows with pre-existing Objects reuse the
  // grouping's buffers once it is done: events (hkeys / hrows), sorted events (orphans /
  // minrow), scan elements (hkeys)
  const size_t m = n + n_seed;
  const size_t b_rep = up256(n * 4), b_hk = up256(m * 8), b_hr = up256(m * 4), b_mr = up256(m * 4),
               b_or = up256(n * 8), b_st = up256((steps_total + 1) * 4), b_ct = up256(steps_total * 8),
               b_bo = d_pre_objects ? up256(pre_blocks(n) * 4) : 0,
               b_tl = d_pre_objects ? up256(segmin_tiles_bytes(n)) : 0,
               b_fl = d_pre_objects ? up256(pre_filter_bytes()) : 0;
  int rc = ensure(c, c->staging,
                  b_rep + b_hk + b_hr + b_mr + b_or + b_st + b_ct + b_bo + b_tl + b_fl + 256);
  if (rc) return rc;
  char* p = (char*)c->staging.p;
  uint32_t* rep = (uint32_t*)p; p += b_rep;
  uint64_t* hkeys = (uint64_t*)p; p += b_hk;
  uint32_t* hrows = (uint32_t*)p; p += b_hr;
  uint32_t* minrow = (uint32_t*)p; p += b_mr;
  uint64_t* orphans = (uint64_t*)p; p += b_or;
  uint32_t* starts = (uint32_t*)p; p += b_st;
  uint32_t* counts = (uint32_t*)p; p += b_ct;
  uint32_t* boff = (uint32_t*)p; p += b_bo;
  uint64_t* tiles = (uint64_t*)p; p += b_tl;
  uint32_t* filter = (uint32_t*)p; p += b_fl;
  // hashed rows | orphan rows | waves with a bad Object id | events
  uint64_t* counters = (uint64_t*)p;
  // 1. grouping over the hashed rows (rep = the key's first row; seeded: the lowest existing
  //    Object id when the key has one — mod.rs:180-198 finds Objects by cas over the whole
  //    library), and the rows that stay orphan after being processed (they steer the cursor)
  std::vector<uint64_t> stay;  // row << 8 | state, ascending
  if (d_state || seeded) {
    uint64_t cnt[3] = {0, 0, 0};
    HIP_TRY(c, hipMemsetAsync(counters, 0, 32, s));
    HIP_TRY(c, links_check_ids(d_seed_objects, n_seed, false, counters + 2, s));
    if (d_pre_objects) HIP_TRY(c, links_check_ids(d_pre_objects, n, true, counters + 2, s));
    HIP_TRY(c, links_split(d_keys, d_state, n, hkeys, hrows, counters, orphans, counters + 1,
                           seeded ? LINKS_ROW_FLAG : 0u, s));
    HIP_TRY(c, hipMemcpyAsync(cnt, counters, 24, hipMemcpyDeviceToHost, s));
    HIP_TRY(c, hipStreamSynchronize(s));
    if (cnt[2])
      return fail(c, SD_CAS_EINVAL, "identifier_links: an existing Object id is >= 2^31");
    stay.resize(cnt[1]);
    if (cnt[1]) {
      HIP_TRY(c, hipMemcpyAsync(stay.data(), orphans, cnt[1] * 8, hipMemcpyDeviceToHost, s));
    }
    if (n_seed) {  // the existing Objects' (cas key, id) pairs after the hashed rows
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
  HIP_TRY(c, hipMemcpyAsync(starts, h_starts.data(), h_starts.size() * 4, hipMemcpyHostToDevice, s));
  // 3. rows that already own an Object (links.hip, sd_links_pre_*): the events — hashed rows
  //    of the reached steps that hold an Object — compacted in row order, sorted stably by key,
  //    and scanned; each hashed row then looks its key up in the decision kernel
  uint64_t n_ev = 0;
  if (d_pre_objects) {
    HIP_TRY(c, links_pre_count(d_state, d_pre_objects, reached, boff, counters + 3, s));
    HIP_TRY(c, hipMemcpyAsync(&n_ev, counters + 3, 8, hipMemcpyDeviceToHost, s));
    HIP_TRY(c, hipStreamSynchronize(s));
  }
  if (n_ev) {
    HIP_TRY(c, hipMemsetAsync(filter, 0, pre_filter_bytes(), s));
    HIP_TRY(c, links_pre_emit(d_keys, d_state, d_pre_objects, reached, boff, hkeys, hrows, filter, s));
    uint64_t* skeys = orphans;
    uint32_t* srows = minrow;
    if ((rc = sd_cas_sort_pairs_dev(c, hkeys, hrows, n_ev, skeys, srows, 0, 64, s))) return rc;
    HIP_TRY(c, links_pre_scan(skeys, srows, d_pre_objects, n_ev, starts, (uint32_t)nsteps, hkeys,
                              tiles, s));
  }
  // 4. per-row decisions + per-step counts (device)
  HIP_TRY(c, hipMemsetAsync(counts, 0, std::max<size_t>(nsteps, 1) * 8, s));
  HIP_TRY(c, links_decide(d_state, rep, n, starts, (uint32_t)nsteps, reached, d_step, d_object,
                          d_action, counts, seeded, d_keys, orphans, minrow, hkeys, filter, n_ev,
                          (uint32_t)chunk, s));
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

int sd_cas_identifier_links_seeded_dev(sd_cas_ctx* c, const uint64_t* d_keys, const uint8_t* d_state,
                                       size_t n, uint32_t chunk, const uint64_t* d_seed_keys,
                                       const uint32_t* d_seed_objects, size_t n_seed, uint32_t* d_step,
                                       uint32_t* d_object, uint8_t* d_action, uint64_t* h_step_counts,
                                       size_t max_steps, uint64_t* out_steps, void* stream) {
  return sd_cas_identifier_links_ex_dev(c, d_keys, d_state, n, chunk, d_seed_keys, d_seed_objects,
                                        n_seed, nullptr, d_step, d_object, d_action, h_step_counts,
                                        max_steps, out_steps, stream);
}

int sd_cas_identifier_links_dev(sd_cas_ctx* c, const uint64_t* d_keys, const uint8_t* d_state,
                                size_t n, uint32_t chunk, uint32_t* d_step, uint32_t* d_object,
                                uint8_t* d_action, uint64_t* h_step_counts, size_t max_steps,
                                uint64_t* out_steps, void* stream) {
  return sd_cas_identifier_links_seeded_dev(c, d_keys, d_state, n, chunk, nullptr, nullptr, 0, d_step,
                                            d_object, d_action, h_step_counts, max_steps, out_steps,
                                            stream);
}

int sd_cas_identifier_links_ex(sd_cas_ctx* c, const uint64_t* h_keys, const uint8_t* h_state,
                               size_t n, uint32_t chunk, const uint64_t* h_seed_keys,
                               const uint32_t* h_seed_objects, size_t n_seed,
                               const uint32_t* h_pre_objects, uint32_t* h_step, uint32_t* h_object,
                               uint8_t* h_action, uint64_t* h_step_counts, size_t max_steps,
                               uint64_t* out_steps) {
  if (!c) return SD_CAS_EINVAL;
  if ((n && (!h_keys || !h_step || !h_object || !h_action)) ||
      (n_seed && (!h_seed_keys || !h_seed_objects)))
    return fail(c, SD_CAS_EINVAL, "identifier_links: bad arguments");
  for (size_t j = 0; j < n_seed; j++)
    if (h_seed_objects[j] >= LINKS_ROW_FLAG)
      return fail(c, SD_CAS_EINVAL, "identifier_links: existing Object id %u >= 2^31", h_seed_objects[j]);
  if (h_pre_objects)
    for (size_t i = 0; i < n; i++)
      if (h_pre_objects[i] >= LINKS_ROW_FLAG && h_pre_objects[i] != SD_CAS_NO_OBJECT)
        return fail(c, SD_CAS_EINVAL, "identifier_links: row %zu's Object id %u >= 2^31", i,
                    h_pre_objects[i]);
  if (n == 0 || n >= (1ull << 32))
    return sd_cas_identifier_links_dev(c, nullptr, nullptr, n, chunk, nullptr, nullptr, nullptr,
                                       h_step_counts, max_steps, out_steps, c->stream);
  HIP_TRY(c, hipSetDevice(c->device));
  // device copies (c->io): keys | state | step | object | action | seed keys | seed ids |
  // pre-existing Objects
  const size_t bk = up256(n * 8), bs = up256(n), b4 = up256(n * 4);
  const size_t bsk = up256(n_seed * 8), bso = up256(n_seed * 4), bpo = h_pre_objects ? b4 : 0;
  int rc = ensure(c, c->io, bk + 2 * bs + 2 * b4 + bsk + bso + bpo);
  if (rc) return rc;
  char* p = (char*)c->io.p;
  uint64_t* d_keys = (uint64_t*)p; p += bk;
  uint8_t* d_state = h_state ? (uint8_t*)p : nullptr; p += bs;
  uint32_t* d_step = (uint32_t*)p; p += b4;
  uint32_t* d_object = (uint32_t*)p; p += b4;
  uint8_t* d_action = (uint8_t*)p; p += bs;
  uint64_t* d_seed_keys = (uint64_t*)p; p += bsk;
  uint32_t* d_seed_objects = (uint32_t*)p; p += bso;
  uint32_t* d_pre = h_pre_objects ? (uint32_t*)p : nullptr;
  hipStream_t s = c->stream;
  HIP_TRY(c, hipMemcpyAsync(d_keys, h_keys, n * 8, hipMemcpyHostToDevice, s));
  if (h_state) HIP_TRY(c, hipMemcpyAsync(d_state, h_state, n, hipMemcpyHostToDevice, s));
  if (n_seed) {
    HIP_TRY(c, hipMemcpyAsync(d_seed_keys, h_seed_keys, n_seed * 8, hipMemcpyHostToDevice, s));
    HIP_TRY(c, hipMemcpyAsync(d_seed_objects, h_seed_objects, n_seed * 4, hipMemcpyHostToDevice, s));
  }
  if (d_pre) HIP_TRY(c, hipMemcpyAsync(d_pre, h_pre_objects, n * 4, hipMemcpyHostToDevice, s));
  rc = sd_cas_identifier_links_ex_dev(c, d_keys, d_state, n, chunk, d_seed_keys, d_seed_objects,
                                      n_seed, d_pre, d_step, d_object, d_action, h_step_counts,
                                      max_steps, out_steps, s);
  if (rc) return rc;
  HIP_TRY(c, hipMemcpyAsync(h_step, d_step, n * 4, hipMemcpyDeviceToHost, s));
  HIP_TRY(c, hipMemcpyAsync(h_object, d_object, n * 4, hipMemcpyDeviceToHost, s));
  HIP_TRY(c, hipMemcpyAsync(h_action, d_action, n, hipMemcpyDeviceToHost, s));
  HIP_TRY(c, hipStreamSynchronize(s));
  return SD_CAS_OK;
}

int sd_cas_identifier_links_seeded(sd_cas_ctx* c, const uint64_t* h_keys, const uint8_t* h_state,
                                   size_t n, uint32_t chunk, const uint64_t* h_seed_keys,
                                   const uint32_t* h_seed_objects, size_t n_seed, uint32_t* h_step,
                                   uint32_t* h_object, uint8_t* h_action, uint64_t* h_step_counts,
                                   size_t max_steps, uint64_t* out_steps) {
  return sd_cas_identifier_links_ex(c, h_keys, h_state, n, chunk, h_seed_keys, h_seed_objects, n_seed,
                                    nullptr, h_step, h_object, h_action, h_step_counts, max_steps,
                                    out_steps);
}

int sd_cas_identifier_links(sd_cas_ctx* c, const uint64_t* h_keys, const uint8_t* h_state,
                            size_t n, uint32_t chunk, uint32_t* h_step, uint32_t* h_object,
                            uint8_t* h_action, uint64_t* h_step_counts, size_t max_steps,
                            uint64_t* out_steps) {
  return sd_cas_identifier_links_seeded(c, h_keys, h_state, n, chunk, nullptr, nullptr, 0, h_step,
                                        h_object, h_action, h_step_counts, max_steps, out_steps);
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
