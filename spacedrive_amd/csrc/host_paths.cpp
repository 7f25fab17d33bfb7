// host_paths.cpp — the host-buffer and path entry points of the C ABI (include/sd_hip_cas.h):
// sd_cas_generate_cas_ids (messages in host memory), sd_cas_generate_cas_ids_from_paths and
// sd_cas_file_metadata_from_paths (FileMetadata::new + generate_cas_id over a job step's
// paths: core/src/object/file_identifier/mod.rs:55-95, core/src/object/cas.rs:23-62 — the
// persistent pread pool at the cas.rs offsets, the streamed single-window pipeline and the
// windowed double-buffered one), sd_cas_hash_sampled_host[_ring] (config 3's PCIe-inclusive
// stream).  Split out of sd_hip_cas.cpp; every digest comes from the HIP kernels.
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
#include <chrono>
#include <memory>
#include <string>
#include <thread>
#include <vector>

#include "sd_checksum.h"
#include "sd_group.h"
#include "sd_kernels.h"
#include "sd_mix.h"

using namespace sdcas;

#include "sd_debug.h"
#include "ctx_internal.h"

// short local names for the shared helpers
#define fail sd_fail
#define pick sd_pick
#define ensure sd_ensure
#define ensure_pinned sd_ensure_pinned

extern "C" {

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
  // Round 6: the last windows TAPER — a window's target is at most half of what remains — so
  // the call's un-overlapped tail (the last full window's H2D + hash after the gather ends;
  // gather and H2D run at about the same rate) shrinks to about two small windows' copies
  // (SD_PATHS_TAPER 0: equal windows, round 5)
#ifndef SD_PATHS_TAPER
#define SD_PATHS_TAPER 1
#endif
  constexpr size_t GATHER_WINDOW = 2048;
  constexpr size_t SMALL_BATCH_FILES = 2048;
  constexpr uint64_t SMALL_BATCH_BYTES = 16ull << 20;
  constexpr uint64_t MIN_WINDOW_BYTES = 2ull << 20;
  std::vector<size_t> wstart{0};
  {
    uint64_t total = 0;
    for (size_t i = 0; i < n; i++) total += up128(lens[i]);
    const bool one_window = n <= SMALL_BATCH_FILES && total <= SMALL_BATCH_BYTES;
    const uint64_t target = one_window ? SMALL_BATCH_BYTES
                                       : std::min<uint64_t>(64ull << 20, std::max<uint64_t>(MIN_WINDOW_BYTES, total / 12));
    auto window_target = [&](uint64_t remaining) {
      return one_window || !SD_PATHS_TAPER ? target
                                           : std::min(target, std::max(MIN_WINDOW_BYTES, remaining / 2));
    };
    uint64_t bytes = 0, left = total, want = window_target(left);
    for (size_t i = 0; i < n; i++) {
      const size_t files = i - wstart.back();
      if (files && (files == GATHER_WINDOW || bytes + up128(lens[i]) > want)) {
        wstart.push_back(i);
        bytes = 0;
        want = window_target(left);
      }
      bytes += up128(lens[i]);
      left -= up128(lens[i]);
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
#ifndef SD_PATHS_CALLER_READS
#define SD_PATHS_CALLER_READS 0
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
      const unsigned k = std::max(1u, std::min(16u, (unsigned)((m + 7) / 8)));
      // (round 6) the readers are all pool threads — bound to the GPU's NUMA node, see
      // sd_cas_ctx_create — and the calling thread only waits; SD_PATHS_CALLER_READS 1: the
      // calling thread reads too (round 5)
      if (SD_PATHS_CALLER_READS || k == 1) c->pool.run(k, worker);
      else c->pool.run2(k, worker, []() {});
      return SD_CAS_OK;
    }
    // streamed: this thread pumps the copies, up to 15 pool threads read (~7 files each for
    // a 100-file step; the job's share of the host is 16 cores)
    const unsigned threads = std::max(1u, std::min(15u, (unsigned)((m + 6) / 7)));
    // the pump: metadata first, then each finished prefix of the content (items are taken
    // in visit order, so a prefix of items is a prefix of the virtual byte space below)
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
  tr.note("windows", (double)nw);
  tr.note("private_threads", (double)c->pool.private_threads());
  if (rc) {
    // a failed call leaves nothing in flight: its pulls (copy streams) and an early
    // whole-file hash (copy2) would otherwise still read the staging, or write keys into it,
    // while the next call gathers into the same buffers
    (void)hipStreamSynchronize(c->copy);
    (void)hipStreamSynchronize(c->copy2);
    (void)hipStreamSynchronize(c->stream);
  }
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
    if (e == hipSuccess) e = sd_dispatch_sampled(c, d_content, stride, d_sizes, m, d_keys, c->stream);
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

}  // extern "C"
