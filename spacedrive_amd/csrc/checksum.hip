// checksum.hip — full-content BLAKE3 of one large file on gfx950 (K3, validator path).
//
// Replaces file_checksum (core/src/object/validation/hash.rs:11-25), which feeds the whole
// file through ONE blake3::Hasher on one thread, 1 MiB at a time, and returns the full
// 64-hex digest.  Here the file is hashed tree-parallel:
//   sd_b3_chunk_groups: 256 lanes x LC chunks per workgroup (iteration j: lane t hashes
//     chunk j*256+t, so each wave load still covers 64 consecutive KiB); chunk CVs go to
//     LDS and the workgroup pair-and-promotes them to ONE subtree CV (8 + log2 LC levels).
//     LC > 1 amortises the reduction's idle lanes: with LC = 1 the upper levels run one
//     mostly idle wave each for 16 wave-compressions of chunk work per wave (~7 % of
//     issue slots); with LC = 4 every lane is busy through the first two levels.
//   sd_b3_reduce_cvs: the same pair-and-promote over 256 CVs at a time, repeated until
//     one CV remains; only the very last parent carries ROOT.
// Level-wise pair-and-promote over aligned groups of 2^k equals BLAKE3's left-balanced
// tree (checked by the oracle's third formulation, blake3_levelwise).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "blake3_device.hpp"
#include "sd_checksum.h"
#include "sd_debug.h"
#include "sd_group.h"

#include <algorithm>

namespace sdcas {

constexpr int GROUP = 256;  // threads per workgroup = CVs per reduce workgroup
#ifndef K3_LANE_CHUNKS
#define K3_LANE_CHUNKS 4   // chunks per lane in sd_b3_chunk_groups (profiles/r01_k3_lc.log)
#endif
constexpr uint64_t GROUP_CHUNKS = (uint64_t)GROUP * K3_LANE_CHUNKS;  // chunks per subtree
static_assert((K3_LANE_CHUNKS & (K3_LANE_CHUNKS - 1)) == 0, "subtrees must be 2^k chunks");

// CV of one FULL 1 KiB chunk (never a root: a one-chunk input takes chunk_cv below), with
// the chunk's first line pair already in A (loaded one chunk ahead), and the
// first pair of the lane's NEXT chunk (`next`, when non-null) loaded into A during this
// chunk's last compressions: 8 line pairs (128-B lines) issued one pair ahead, ping-ponged
// in registers like K1.  A lane's chunks are 256 KiB apart; without the cross-chunk
// prefetch every chunk started with a full HBM load latency before its first compression.
__device__ __forceinline__ void full_chunk_cv_pf(const uint4* __restrict__ q, const uint4* __restrict__ next,
                                                 uint64_t ctr, uint32_t (&cv)[8], uint4 (&A)[8]) {
  set_iv(cv);
  uint4 B[8];
#pragma unroll 1
  for (uint32_t p = 0; p < 8; p += 2) {
#pragma unroll
    for (int i = 0; i < 8; ++i) B[i] = q[8u * (p + 1) + i];
    {
      const uint32_t m[16] = {A[0].x, A[0].y, A[0].z, A[0].w, A[1].x, A[1].y, A[1].z, A[1].w,
                              A[2].x, A[2].y, A[2].z, A[2].w, A[3].x, A[3].y, A[3].z, A[3].w};
      compress(cv, m, (uint32_t)ctr, (uint32_t)(ctr >> 32), BLOCK_LEN, p == 0 ? (uint32_t)CHUNK_START : 0u);
    }
    {
      const uint32_t m[16] = {A[4].x, A[4].y, A[4].z, A[4].w, A[5].x, A[5].y, A[5].z, A[5].w,
                              A[6].x, A[6].y, A[6].z, A[6].w, A[7].x, A[7].y, A[7].z, A[7].w};
      compress(cv, m, (uint32_t)ctr, (uint32_t)(ctr >> 32), BLOCK_LEN, 0u);
    }
    // the next pair of this chunk, or the first pair of the lane's next chunk
    const uint4* src = p + 2 < 8 ? q + 8u * (p + 2) : next;
    if (src) {
#pragma unroll
      for (int i = 0; i < 8; ++i) A[i] = src[i];
    }
    {
      const uint32_t m[16] = {B[0].x, B[0].y, B[0].z, B[0].w, B[1].x, B[1].y, B[1].z, B[1].w,
                              B[2].x, B[2].y, B[2].z, B[2].w, B[3].x, B[3].y, B[3].z, B[3].w};
      compress(cv, m, (uint32_t)ctr, (uint32_t)(ctr >> 32), BLOCK_LEN, 0u);
    }
    {
      const uint32_t m[16] = {B[4].x, B[4].y, B[4].z, B[4].w, B[5].x, B[5].y, B[5].z, B[5].w,
                              B[6].x, B[6].y, B[6].z, B[6].w, B[7].x, B[7].y, B[7].z, B[7].w};
      compress(cv, m, (uint32_t)ctr, (uint32_t)(ctr >> 32), BLOCK_LEN,
               p == 6 ? (uint32_t)CHUNK_END : 0u);
    }
  }
}

// CV (or ROOT digest) of one chunk of `clen` <= 1024 bytes at global chunk index `ctr`
// (the input's last chunk; partial or empty).  Quads past the end are re-pointed at quad 0
// (in bounds) and the final block is masked, as in K2.
__device__ __forceinline__ void chunk_cv(const uint4* __restrict__ q, uint32_t clen, uint64_t ctr,
                                         bool root, uint32_t (&cv)[8]) {
  const uint32_t nblk = clen == 0 ? 1u : (clen + 63u) >> 6;
  set_iv(cv);
  const uint4 z = make_uint4(0u, 0u, 0u, 0u);
  uint4 a0 = z, a1 = z, a2 = z, a3 = z;  // an empty input reads nothing (its round-up is 0 B)
  auto load = [&](uint32_t b) {
    const uint32_t o = b << 6;
    a0 = q[(o < clen) ? 4 * b : 0u];
    a1 = q[(o + 16u < clen) ? 4 * b + 1 : 0u];
    a2 = q[(o + 32u < clen) ? 4 * b + 2 : 0u];
    a3 = q[(o + 48u < clen) ? 4 * b + 3 : 0u];
  };
  if (clen) load(0);
  for (uint32_t b = 0; b < nblk; ++b) {
    uint32_t m[16] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w,
                      a2.x, a2.y, a2.z, a2.w, a3.x, a3.y, a3.z, a3.w};
    const uint32_t rem = clen - (b << 6);
    const uint32_t blen = clen == 0 ? 0u : (rem < 64u ? rem : 64u);
    if (blen < 64u) {
#pragma unroll
      for (int w = 0; w < 16; ++w) {
        const int vb = (int)blen - 4 * w;
        m[w] &= vb >= 4 ? 0xFFFFFFFFu : (vb <= 0 ? 0u : ((1u << (8 * vb)) - 1u));
      }
    }
    if (b + 1 < nblk) load(b + 1);
    uint32_t flags = (b == 0 ? (uint32_t)CHUNK_START : 0u) | (b + 1 == nblk ? (uint32_t)CHUNK_END : 0u);
    if (root && b + 1 == nblk) flags |= ROOT;
    compress(cv, m, (uint32_t)ctr, (uint32_t)(ctr >> 32), blen, flags);
  }
}

// Pair-and-promote `count` (<= PER * 256) CVs held in LDS cvs[][8] down to one (in cvs[0]).
// `root_last`: the final parent carries ROOT (only when this is the whole tree's top).
// Thread t computes the parents t, t+256, ... of a level; all reads of a level finish
// before its writes (parent p overwrites slot p, which another thread's pair may read).
template <int PER>
__device__ __forceinline__ void lds_reduce(uint32_t (*cvs)[8], uint32_t count, bool root_last) {
  const uint32_t t = threadIdx.x;
  while (count > 1) {
    const uint32_t pairs = count >> 1;
    const bool odd = count & 1u;
    uint32_t out[PER][8];
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      const uint32_t p = t + (uint32_t)k * GROUP;
      if (p < pairs) {
        uint32_t l[8], r[8];
#pragma unroll
        for (int w = 0; w < 8; ++w) { l[w] = cvs[2 * p][w]; r[w] = cvs[2 * p + 1][w]; }
        parent(out[k], l, r, (root_last && count == 2) ? (uint32_t)ROOT : 0u);
      } else if (odd && p == pairs) {
#pragma unroll
        for (int w = 0; w < 8; ++w) out[k][w] = cvs[count - 1][w];
      }
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      const uint32_t p = t + (uint32_t)k * GROUP;
      if (p < pairs || (odd && p == pairs)) {
#pragma unroll
        for (int w = 0; w < 8; ++w) cvs[p][w] = out[k][w];
      }
    }
    __syncthreads();
    count = pairs + (odd ? 1u : 0u);
  }
}

// Chunks [g*GC, g*GC+GC) of the buffer (global chunk index chunk0 + ...) -> their subtree
// CV in out8[0..8); when the buffer has one group and root_if_single_group, the ROOT digest
// (a single chunk is then the root itself).  Called by the whole workgroup; leaves cvs free.
template <int LC>
__device__ __forceinline__ void group_subtree(const uint8_t* __restrict__ data, uint64_t len,
                                              uint64_t chunk0, uint64_t g, uint32_t* __restrict__ out8,
                                              int root_if_single_group, uint32_t (*cvs)[8]) {
  constexpr uint32_t GC = GROUP * LC;
  const uint64_t nchunks = len == 0 ? 1 : (len + 1023) >> 10;
  const uint64_t first = g * GC;
  const uint32_t count = (uint32_t)min((uint64_t)GC, nchunks - first);
  const uint32_t t = threadIdx.x;
  const bool whole_tree = root_if_single_group && nchunks <= (uint64_t)GC;
  // a lane's FULL chunks (never the input's last, never a one-chunk input) run with their
  // first line pair loaded one chunk ahead (full_chunk_cv_pf); the rest take chunk_cv
  auto full = [&](uint32_t i) {
    return i < count && first + i + 1 < nchunks;  // not the last chunk: 1,024 bytes
  };
  uint4 A[8];
  if (full(t)) {
    const uint4* q0 = reinterpret_cast<const uint4*>(data + ((first + t) << 10));
#pragma unroll
    for (int k = 0; k < 8; ++k) A[k] = q0[k];
  }
#pragma unroll 1
  for (uint32_t j = 0; j < LC; ++j) {
    const uint32_t i = j * GROUP + t;
    if (i < count) {
      const uint64_t c = first + i;
      const uint64_t off = c << 10;
      uint32_t cv[8];
      if (full(i)) {
        const uint32_t in = i + GROUP;
        const uint4* next = j + 1 < LC && full(in) ? reinterpret_cast<const uint4*>(data + ((first + in) << 10))
                                                   : nullptr;
        full_chunk_cv_pf(reinterpret_cast<const uint4*>(data + off), next, chunk0 + c, cv, A);
      } else {
        chunk_cv(reinterpret_cast<const uint4*>(data + off), (uint32_t)min((uint64_t)1024, len - off),
                 chunk0 + c, whole_tree && nchunks == 1, cv);
      }
#pragma unroll
      for (int w = 0; w < 8; ++w) cvs[i][w] = cv[w];
    }
  }
  __syncthreads();
  lds_reduce<(LC + 1) / 2>(cvs, count, whole_tree);
  if (t < 8) out8[t] = cvs[0][t];
  __syncthreads();  // cvs[0] read before the caller's next group overwrites it
}

// One workgroup per group of the buffer: out[8 g ..] = subtree CV of group g.
template <int LC>
__device__ __forceinline__ void chunk_groups(const uint8_t* __restrict__ data, uint64_t len,
                                             uint64_t chunk0, uint32_t* __restrict__ out,
                                             int root_if_single_group, uint32_t (*cvs)[8]) {
  group_subtree<LC>(data, len, chunk0, blockIdx.x, out + (uint64_t)blockIdx.x * 8,
                    root_if_single_group, cvs);
}

extern "C" __global__ void __launch_bounds__(GROUP)
sd_b3_chunk_groups(const uint8_t* __restrict__ data, uint64_t len, uint64_t chunk0,
                   uint32_t* __restrict__ out, int root_if_single_group) {
  __shared__ uint32_t cvs[GROUP * K3_LANE_CHUNKS][8];
  chunk_groups<K3_LANE_CHUNKS>(data, len, chunk0, out, root_if_single_group, cvs);
}

// Reduce groups of 256 CVs: in[cnt][8] -> out[ceil(cnt/256)][8].
extern "C" __global__ void __launch_bounds__(GROUP)
sd_b3_reduce_cvs(const uint32_t* __restrict__ in, uint64_t cnt, uint32_t* __restrict__ out,
                 int root_if_single_group) {
  __shared__ uint32_t cvs[GROUP][8];
  const uint64_t first = (uint64_t)blockIdx.x * GROUP;
  const uint32_t count = (uint32_t)min((uint64_t)GROUP, cnt - first);
  const uint32_t t = threadIdx.x;
  if (t < count) {
#pragma unroll
    for (int w = 0; w < 8; ++w) cvs[t][w] = in[(first + t) * 8 + w];
  }
  __syncthreads();
  lds_reduce<1>(cvs, count, root_if_single_group && cnt <= (uint64_t)GROUP);
  if (t < 8) out[(uint64_t)blockIdx.x * 8 + t] = cvs[0][t];
}

// ---- many buffers per launch chain (the validator job over a location) -------------------
// validator_job.rs:107-172 runs one file_checksum (hash.rs:11-25) per job step; here a
// batch of n buffers is hashed by ONE chain of launches, split by size:
//   small buffers (<= SMALL_CHUNKS KiB, documents): ONE WAVE per buffer — lane c hashes
//     chunk c, the wave pair-and-promotes its chunk CVs in its own LDS slice (no workgroup
//     barrier), 4 buffers per workgroup in flight;
//   larger buffers: cut into the same 1 MiB subtree groups (GROUP_CHUNKS chunks) as K3;
//     their groups form one work list (gstart = exclusive scan of the per-buffer group
//     counts, owner[item] = the buffer of work item `item`) that a large grid strides over:
//       sd_b3_batch_groups: item -> its subtree CV, or the buffer's ROOT digest directly
//         when the buffer has a single group;
//       sd_b3_batch_blocks + sd_b3_batch_reduce: the buffers with >= 2 groups: aligned
//         blocks of 256 group CVs pair-and-promote to one CV each in LDS, one workgroup per
//         block (a buffer of up to 65,536 groups = 64 GiB has <= 256 blocks), then one
//         workgroup per buffer takes those to the ROOT digest — the level-wise tree of K3's
//         reduce_to_one.
constexpr uint32_t BATCH_MAX_GROUPS = GROUP * GROUP;  // 64 GiB per buffer
constexpr uint32_t SMALL_CHUNKS = 64;                 // a wave's lanes
constexpr uint32_t MID_CHUNKS = 256;                  // a wave's lanes x 4 chunks
constexpr uint64_t BATCH_MAX_LEN = (uint64_t)BATCH_MAX_GROUPS * GROUP_CHUNKS * 1024;

__device__ __forceinline__ uint64_t chunks_of(uint64_t len) { return len == 0 ? 1 : (len + 1023) >> 10; }

// ---- the lane-per-buffer class (sd_b3_batch_lane below) --------------------------------
#ifndef LANE_MAX_CHUNKS
#define LANE_MAX_CHUNKS 128
#endif
#ifndef LANE_MIN_BUFFERS
#define LANE_MIN_BUFFERS 65536
#endif
constexpr uint32_t LANE_CHUNKS = LANE_MAX_CHUNKS;
static_assert(LANE_CHUNKS >= SMALL_CHUNKS && LANE_CHUNKS <= MID_CHUNKS &&
                  (LANE_CHUNKS & (LANE_CHUNKS - 1)) == 0,
              "the lane class replaces the segment kernels' classes");
// The lane kernel takes the lane-class buffers of at most `cut` chunks; the segment / mid
// kernels the rest.  A lane of c chunks runs c x 17 compressions back to back, so a few
// long buffers in a batch of short ones would make a tail far longer than the whole
// batch's share of the chip: cut = min(LANE_CHUNKS, LANE_TAIL x the class's total chunks /
// LANE_SLOTS) keeps the longest lane within LANE_TAIL x the time the class needs at full
// occupancy (LANE_SLOTS lanes: 256 CUs x 4 SIMDs x 2 waves x 64).  Measured
// (profiles/r02b_lane_ab_pass4/): 65,536 buffers, 8 % of them 96-128 KiB: no cut 2.86 ms,
// segment kernels only 1.07, cut 0.87; LANE_TAIL 1 and 2 split uniform batches between two
// serial kernels (65,536 x U(0, 16) KiB: 0.70-0.77 vs 0.54 ms), 4 does not.
#ifndef LANE_TAIL
#define LANE_TAIL 4
#endif
constexpr uint64_t LANE_SLOTS = 256ull * 4 * 2 * 64;
// With the lane path the batch is visited in one stable order by descending chunk count
// (sd_b3_lane_keys + one radix sort): positions [0, info[1]) hold the 65..256-chunk
// buffers, then info[2] of 17..64 chunks, then info[3] of <= 16, then the rest (over
// MID_CHUNKS, or refused); info[0] = the lane class's chunk count.  Each segment / mid kernel
// walks its own range of positions and stops at the first buffer the lane kernel takes.
struct LaneInfo {
  const uint32_t* order;  // nullptr: no lane path, positions = buffer indices
  const uint32_t* info;
};
__device__ __forceinline__ uint32_t lane_cut(const uint32_t* __restrict__ info) {
  if (!info) return 0u;
  const uint64_t c = (uint64_t)LANE_TAIL * info[0] / LANE_SLOTS;
  return (uint32_t)(c < LANE_CHUNKS ? c : LANE_CHUNKS);
}
// positions [lo, hi) of the class ending at SEG chunks (16, 64 or MID_CHUNKS)
template <uint32_t SEG>
__device__ __forceinline__ void lane_range(const uint32_t* __restrict__ info, uint64_t n,
                                           uint64_t& lo, uint64_t& hi) {
  if (!info) { lo = 0; hi = n; return; }
  const uint64_t m = info[1], s64 = info[2], s16 = info[3];
  lo = SEG == MID_CHUNKS ? 0 : SEG == SMALL_CHUNKS ? m : m + s64;
  hi = SEG == MID_CHUNKS ? m : SEG == SMALL_CHUNKS ? m + s64 : m + s64 + s16;
}

// A buffer is hashed only if it is 16-B aligned and ends within the arena (a bad offset or
// length is reported, not read out of bounds).
__device__ __forceinline__ bool buffer_ok(uint64_t off, uint64_t len, uint64_t arena_bytes) {
  return (off & 15) == 0 && len <= arena_bytes && off <= arena_bytes - len && len <= BATCH_MAX_LEN;
}

// per-buffer group counts for the big-buffer work list (0 for small and for rejected
// buffers); *bad |= 1 for a buffer over 64 GiB, 4 for one outside the arena or misaligned
extern "C" __global__ void __launch_bounds__(256)
sd_b3_batch_count(const uint64_t* __restrict__ offs, const uint64_t* __restrict__ lens, uint64_t n,
                  uint64_t arena_bytes, uint32_t* __restrict__ groups, uint32_t* __restrict__ bad,
                  uint32_t* __restrict__ lane_info) {
  const uint64_t f = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (f < 4 && lane_info) lane_info[f] = 0u;  // sd_b3_lane_keys accumulates them next
  if (f >= n) return;
  const uint64_t len = lens[f];
  const uint64_t nch = chunks_of(len);
  const bool ok = buffer_ok(offs[f], len, arena_bytes);
  if (!ok) atomicOr(bad, len > BATCH_MAX_LEN ? 1u : 4u);
  groups[f] = nch <= MID_CHUNKS || !ok ? 0u : (uint32_t)((nch + GROUP_CHUNKS - 1) / GROUP_CHUNKS);
}

// owner[item] = the last f with gstart[f] <= item (every listed buffer owns >= 1 item)
extern "C" __global__ void __launch_bounds__(256)
sd_b3_batch_owner(const uint32_t* __restrict__ gstart, const unsigned long long* __restrict__ gtotal,
                  uint64_t n, uint64_t items_cap, uint32_t* __restrict__ owner) {
  const uint64_t total = *gtotal;
  if (total > items_cap) return;  // overlapping buffers: the list does not fit (reported below)
  const uint64_t lim = total;
  for (uint64_t item = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; item < lim;
       item += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t lo = 0, hi = n;  // gstart[lo] <= item < gstart[hi] (gstart[n] = total)
    while (hi - lo > 1) {
      const uint64_t mid = (lo + hi) >> 1;
      if (gstart[mid] <= item) lo = mid; else hi = mid;
    }
    // the search needs a monotone gstart: item inside its owner's range
    SD_DBG_CHECK(gstart[lo] <= item && (lo + 1 == n || item < gstart[lo + 1]),
                 "batch owner: item %llu -> buffer %llu [%u, %u)", (unsigned long long)item,
                 (unsigned long long)lo, gstart[lo], lo + 1 < n ? gstart[lo + 1] : (uint32_t)total);
    owner[item] = (uint32_t)lo;
  }
}

// wave-synchronous LDS phases of the small-buffer path (one wave per buffer: no workgroup
// barrier, only ordering of this wave's own LDS accesses)
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

// One buffer per SEG-lane segment (SEG = 16: buffers of <= 16 chunks, 4 per wave; SEG = 64:
// 17..64 chunks, one per wave): lane l of the segment hashes chunk l, and the segment
// pair-and-promotes its chunk CVs in its own LDS slice, log2(SEG) fixed levels run by the
// whole wave in step (segments whose tree is done idle through the rest).
template <uint32_t SEG>
__device__ __forceinline__ void batch_small_body(const uint8_t* __restrict__ arena,
                                                 uint64_t arena_bytes,
                                                 const uint64_t* __restrict__ offs,
                                                 const uint64_t* __restrict__ lens, uint64_t n,
                                                 uint32_t* __restrict__ digests,
                                                 uint32_t (*cvs)[8], LaneInfo li) {
  constexpr uint32_t PER_WAVE = 64 / SEG;
  const uint32_t cut = lane_cut(li.info);
  uint64_t lo, hi;
  lane_range<SEG>(li.info, n, lo, hi);
  constexpr uint32_t LOW = SEG == 64 ? 16 : 0;  // this class: LOW < chunks <= SEG
  const uint32_t lane = threadIdx.x & 63u, seg = lane / SEG, sl = lane % SEG;
  uint32_t (*mine)[8] = cvs + (threadIdx.x >> 6) * 64 + seg * SEG;  // the segment's slice
  const uint64_t slots = (uint64_t)gridDim.x * (blockDim.x / 64) * PER_WAVE;
  const uint64_t first = ((uint64_t)blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6)) * PER_WAVE + seg;
  for (uint64_t base = lo + first - seg; base < hi; base += slots) {  // wave-uniform trips
    if (li.order && chunks_of(lens[li.order[base]]) <= cut) break;  // the wave's longest: the
                                                                      // rest go one per lane
    const uint64_t t = base + seg;
    const uint64_t f = t < hi ? (li.order ? li.order[t] : t) : n;
    const uint64_t len = f < n ? lens[f] : 0;
    const uint64_t nch = chunks_of(len);
    const bool mine_class = f < n && nch > LOW && nch > cut && nch <= SEG && buffer_ok(offs[f], len, arena_bytes);
    const uint32_t count = mine_class ? (uint32_t)nch : 0u;
    if (sl < count) {
      const uint64_t off = (uint64_t)sl << 10;
      const uint32_t clen = (uint32_t)min((uint64_t)1024, len - min(len, off));
      uint32_t cv[8];
      // the generic chunk loop for every lane (a full-chunk fast path would diverge from
      // the buffer's partial last chunk inside the wave)
      chunk_cv(reinterpret_cast<const uint4*>(arena + offs[f] + off), clen, sl, count == 1, cv);
      if (count == 1) {
#pragma unroll
        for (int k = 0; k < 8; ++k) digests[8 * f + k] = cv[k];
      } else {
#pragma unroll
        for (int k = 0; k < 8; ++k) mine[sl][k] = cv[k];
      }
    }
    wave_sync();
    uint32_t c = count;
#pragma unroll 1
    for (uint32_t lvl = 1; lvl < SEG; lvl <<= 1) {
      const uint32_t pairs = c >> 1;
      const bool odd = c & 1u;
      const bool work = c > 1 && (sl < pairs || (odd && sl == pairs));
      uint32_t out[8];
      if (c > 1 && sl < pairs) {
        uint32_t l[8], r[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) { l[k] = mine[2 * sl][k]; r[k] = mine[2 * sl + 1][k]; }
        parent(out, l, r, c == 2 ? (uint32_t)ROOT : 0u);
      } else if (work) {
#pragma unroll
        for (int k = 0; k < 8; ++k) out[k] = mine[c - 1][k];
      }
      wave_sync();
      if (work) {
#pragma unroll
        for (int k = 0; k < 8; ++k) mine[sl][k] = out[k];
      }
      wave_sync();
      if (c > 1) c = pairs + (odd ? 1u : 0u);
    }
    if (count > 1 && sl < 8) digests[8 * f + sl] = mine[0][sl];
    wave_sync();  // mine[0] read before the next buffer's chunk CVs overwrite it
  }
}

extern "C" __global__ void __launch_bounds__(256)
sd_b3_batch_small16(const uint8_t* __restrict__ arena, uint64_t arena_bytes,
                    const uint64_t* __restrict__ offs, const uint64_t* __restrict__ lens, uint64_t n,
                    const uint32_t* __restrict__ order, const uint32_t* __restrict__ lane_info,
                    uint32_t* __restrict__ digests) {
  __shared__ uint32_t cvs[4 * 64][8];
  batch_small_body<16>(arena, arena_bytes, offs, lens, n, digests, cvs, LaneInfo{order, lane_info});
}

extern "C" __global__ void __launch_bounds__(256)
sd_b3_batch_small64(const uint8_t* __restrict__ arena, uint64_t arena_bytes,
                    const uint64_t* __restrict__ offs, const uint64_t* __restrict__ lens, uint64_t n,
                    const uint32_t* __restrict__ order, const uint32_t* __restrict__ lane_info,
                    uint32_t* __restrict__ digests) {
  __shared__ uint32_t cvs[4 * 64][8];
  batch_small_body<64>(arena, arena_bytes, offs, lens, n, digests, cvs, LaneInfo{order, lane_info});
}

// Buffers of 65..256 chunks (64-256 KiB): ONE WAVE per buffer with CPL = 2 or 4 consecutive
// chunks per lane (lane l: chunks [l CPL, (l+1) CPL), an aligned subtree merged in registers),
// then the lanes' subtree CVs pair-and-promote in the wave's LDS slice — level-wise over
// aligned power-of-two groups, i.e. BLAKE3's left-balanced tree.  In a 1 MiB group
// workgroup (the path above 256 chunks) such a buffer kept 25-100 of 256 lanes busy.
extern "C" __global__ void __launch_bounds__(256)
sd_b3_batch_mid(const uint8_t* __restrict__ arena, uint64_t arena_bytes,
                const uint64_t* __restrict__ offs, const uint64_t* __restrict__ lens, uint64_t n,
                const uint32_t* __restrict__ order, const uint32_t* __restrict__ lane_info,
                uint32_t* __restrict__ digests) {
  __shared__ uint32_t wcv[4 * 64][8];
  const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
  uint32_t (*mine)[8] = wcv + w * 64;
  const uint64_t waves = (uint64_t)gridDim.x * 4;
  const uint32_t cut = lane_cut(lane_info);
  uint64_t lo, hi;
  lane_range<MID_CHUNKS>(lane_info, n, lo, hi);
  for (uint64_t t = lo + (uint64_t)blockIdx.x * 4 + w; t < hi; t += waves) {
    const uint64_t f = order ? order[t] : t;
    const uint64_t len = lens[f];
    const uint64_t nch = chunks_of(len);
    if (order && nch <= cut) break;  // sorted: every later buffer goes one per lane
    // this class: SMALL_CHUNKS < nch <= MID_CHUNKS, less those the lane kernel takes
    if (nch <= SMALL_CHUNKS || nch <= cut || nch > MID_CHUNKS || !buffer_ok(offs[f], len, arena_bytes)) continue;
    const uint32_t cpl = nch <= 128 ? 2u : 4u;               // wave-uniform
    const uint32_t count = (uint32_t)((nch + cpl - 1) / cpl);  // lanes holding a subtree
    const uint8_t* data = arena + offs[f];
    if (lane < count) {
      uint32_t cv[8], acc[8], pend[8];
      uint32_t have = 0;  // subtrees pending: pend (2 chunks) for cpl 4
      for (uint32_t k = 0; k < cpl; ++k) {
        const uint64_t c = (uint64_t)lane * cpl + k;
        if (c >= nch) break;
        const uint64_t off = c << 10;
        const uint32_t clen = (uint32_t)min((uint64_t)1024, len - off);
        chunk_cv(reinterpret_cast<const uint4*>(data + off), clen, c, false, cv);
        if ((k & 1u) == 0) {
#pragma unroll
          for (int q = 0; q < 8; ++q) acc[q] = cv[q];
        } else {
          parent(acc, acc, cv, 0u);  // chunks 2j, 2j+1 -> their parent
          if (k == 3) {
            parent(acc, pend, acc, 0u);  // (0,1), (2,3) -> the lane's 4-chunk subtree
            have = 0;
          } else if (cpl == 4) {
#pragma unroll
            for (int q = 0; q < 8; ++q) pend[q] = acc[q];
            have = 1;
          }
        }
      }
      // a partial last group (the buffer's end): pend (chunks 0,1) + acc (chunk 2) -> parent
      const uint32_t got = (uint32_t)min((uint64_t)cpl, nch - (uint64_t)lane * cpl);
      if (cpl == 4 && got == 3) parent(acc, pend, acc, 0u);
      else if (cpl == 4 && got == 2 && have) {
#pragma unroll
        for (int q = 0; q < 8; ++q) acc[q] = pend[q];
      }
#pragma unroll
      for (int q = 0; q < 8; ++q) mine[lane][q] = acc[q];
    }
    wave_sync();
#pragma unroll 1
    for (uint32_t c = count; c > 1;) {
      const uint32_t pairs = c >> 1;
      const bool odd = c & 1u;
      uint32_t out[8];
      if (lane < pairs) {
        uint32_t l[8], r[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) { l[q] = mine[2 * lane][q]; r[q] = mine[2 * lane + 1][q]; }
        parent(out, l, r, c == 2 ? (uint32_t)ROOT : 0u);
      } else if (odd && lane == pairs) {
#pragma unroll
        for (int q = 0; q < 8; ++q) out[q] = mine[c - 1][q];
      }
      wave_sync();
      if (lane < pairs || (odd && lane == pairs)) {
#pragma unroll
        for (int q = 0; q < 8; ++q) mine[lane][q] = out[q];
      }
      wave_sync();
      c = pairs + (odd ? 1u : 0u);
    }
    if (lane < 8) digests[8 * f + lane] = mine[0][lane];
    wave_sync();
  }
}

// ---- ONE BUFFER PER LANE (batches of many small buffers) -------------------------------
// A batch of >= LANE_MIN_BUFFERS buffers has enough of them to fill the chip one per lane
// (those of <= lane_cut() chunks: a few long buffers stay on the kernels above),
// K2's shape: every lane walks its own buffer (128-B line loads, one line ahead), full
// chunks on a fixed 16-block schedule, only the last chunk generic, the CV stack's bottom
// entry in VGPRs and the rest in an LDS column per lane.  Buffers are visited by
// descending chunk count (one stable radix pass, sd_b3_lane_keys), so a wave's lanes share
// their trip counts and same-count buffers keep their arena order.  The segment kernels
// above spend lanes on the pair-and-promote levels and on buffers shorter than their
// segment; they stay for smaller batches, where one buffer per lane would leave the chip
// idle and the per-buffer latency is ~nch x 17 compressions instead of ~16 + log2(nch).
constexpr int ilog2c(uint32_t x) { return x <= 1 ? 0 : 1 + ilog2c(x >> 1); }
// popcount(c) <= log2(LANE_CHUNKS) pending subtrees after c < LANE_CHUNKS chunks; the
// bottom one in VGPRs: 6 x 32 B x 256 lanes = 48 KiB per workgroup for 128 chunks.
// Occupancy is capped at 2 waves per SIMD by LANE_LDS_PAD bytes of dynamic LDS at launch
// (80 KiB per workgroup, 2 per CU): every lane streams its own buffer, and fewer concurrent
// streams run faster (profiles/r02b_lane_ab*: 4 waves/SIMD (64-chunk class) < 3 < 2 > 1;
// docs 1.82 / 2.50 / 2.71 / 2.63 TB/s; a 512-lane workgroup (2 waves, 1 per CU) 2.61).
constexpr int LANE_LDS_DEPTH = ilog2c(LANE_CHUNKS) - 1;
constexpr int LANE_BLOCK = 256;
#ifndef SD_LANE_WAVES
#define SD_LANE_WAVES 2  // waves per SIMD = 256-lane workgroups per CU (LDS-limited)
#endif
constexpr size_t LANE_LDS_PAD = (160u << 10) / SD_LANE_WAVES - sizeof(uint32_t) * LANE_LDS_DEPTH * 8 * LANE_BLOCK;
static_assert((160u << 10) / SD_LANE_WAVES >= sizeof(uint32_t) * LANE_LDS_DEPTH * 8 * LANE_BLOCK,
              "the lane stack fits the workgroup's LDS share");
// The lane class's visiting key: the chunk count, or (block_key) the exact 64-B block count,
// so a wave's lanes share the last chunk's length too.  The block key ran 4 % faster on 1M
// U(0, 16) KiB buffers (3.24 vs 3.37 ms) but 2.4x slower on 262,144 U(1, 128) KiB ones (14.9
// vs 6.2 ms): small block buckets scatter a wave over the arena (profiles/r04_ab_keys.log).
// checksum_batch_device takes it when the arena averages <= LANE_BLOCK_KEY_MEAN bytes per
// buffer (round 5).
constexpr uint64_t LANE_BLOCK_KEY_MEAN = 16384;
constexpr int LANE_KEY_BITS_BLOCKS = ilog2c(MID_CHUNKS * 16) + 1;  // 0..4,096: 13 bits
constexpr int LANE_KEY_BITS_CHUNKS = ilog2c(MID_CHUNKS) + 1;       // 0..256: 9 bits

struct LaneStack {
  uint32_t (*s)[8][LANE_BLOCK];
  uint32_t t;
  uint32_t sp = 0;
  uint32_t bottom[8];
  __device__ __forceinline__ void push(const uint32_t (&cv)[8]) {
    if (sp == 0) {
#pragma unroll
      for (int w = 0; w < 8; ++w) bottom[w] = cv[w];
    } else {
#pragma unroll
      for (int w = 0; w < 8; ++w) s[sp - 1][w][t] = cv[w];
    }
    ++sp;
  }
  __device__ __forceinline__ void pop(uint32_t (&out)[8]) {
    --sp;
    if (sp == 0) {
#pragma unroll
      for (int w = 0; w < 8; ++w) out[w] = bottom[w];
    } else {
#pragma unroll
      for (int w = 0; w < 8; ++w) out[w] = s[sp - 1][w][t];
    }
  }
};

// line P of the buffer (quads 8P..8P+7); all 8 quads are in bounds
__device__ __forceinline__ void lane_line(const uint4* __restrict__ q, uint32_t P, uint4 (&buf)[8]) {
#pragma unroll
  for (int i = 0; i < 8; ++i) buf[i] = q[8u * P + i];
}
// the same with quads at or past the 16-B round-up of len re-pointed at quad 0 (len > 0);
// their bytes only reach the final block, which is masked
__device__ __forceinline__ void lane_line_clamped(const uint4* __restrict__ q, uint32_t P,
                                                  uint32_t len, uint4 (&buf)[8]) {
  const uint32_t b0 = P << 7;
#pragma unroll
  for (int i = 0; i < 8; ++i) buf[i] = q[(b0 + 16u * i < len) ? 8u * P + i : 0u];
}
__device__ __forceinline__ void lane_compress_line(uint32_t (&cv)[8], const uint4 (&A)[8],
                                                   uint32_t ctr, uint32_t f0, uint32_t f1) {
  {
    const uint32_t m[16] = {A[0].x, A[0].y, A[0].z, A[0].w, A[1].x, A[1].y, A[1].z, A[1].w,
                            A[2].x, A[2].y, A[2].z, A[2].w, A[3].x, A[3].y, A[3].z, A[3].w};
    compress(cv, m, ctr, 0u, BLOCK_LEN, f0);
  }
  {
    const uint32_t m[16] = {A[4].x, A[4].y, A[4].z, A[4].w, A[5].x, A[5].y, A[5].z, A[5].w,
                            A[6].x, A[6].y, A[6].z, A[6].w, A[7].x, A[7].y, A[7].z, A[7].w};
    compress(cv, m, ctr, 0u, BLOCK_LEN, f1);
  }
}

// CV of full chunk c (not the buffer's last): A holds line 8c on entry and line 8(c+1)
// (clamped: the next chunk may be the partial last one) on exit; the lines ping-pong
// between A and B with no register moves.
__device__ __forceinline__ void lane_full_chunk(const uint4* __restrict__ q, uint32_t len, uint32_t c,
                                                uint32_t (&cv)[8], uint4 (&A)[8], uint4 (&B)[8]) {
  set_iv(cv);
#pragma unroll 1
  for (uint32_t pp = 0; pp < 3; ++pp) {
    const uint32_t P = 8u * c + 2u * pp;
    lane_line(q, P + 1, B);
    lane_compress_line(cv, A, c, pp == 0 ? (uint32_t)CHUNK_START : 0u, 0u);
    lane_line(q, P + 2, A);
    lane_compress_line(cv, B, c, 0u, 0u);
  }
  lane_line(q, 8u * c + 7u, B);
  lane_compress_line(cv, A, c, 0u, 0u);
  lane_line_clamped(q, 8u * c + 8u, len, A);
  lane_compress_line(cv, B, c, 0u, CHUNK_END);
}

// BLAKE3 digest of buffer q[0, len), len <= LANE_CHUNKS KiB, into cv
__device__ __forceinline__ void lane_digest(const uint4* __restrict__ q, uint32_t len, LaneStack& stk,
                                            uint32_t (&cv)[8]) {
  const uint32_t nch = len == 0 ? 1u : (len + 1023u) >> 10;
  uint4 A[8], B[8];
  if (len) {
    lane_line_clamped(q, 0, len, A);
  } else {  // an empty buffer reads nothing (its round-up is 0 bytes)
#pragma unroll
    for (int i = 0; i < 8; ++i) A[i] = make_uint4(0u, 0u, 0u, 0u);
  }
  for (uint32_t c = 0; c + 1 < nch; ++c) {
    lane_full_chunk(q, len, c, cv, A, B);
    for (uint32_t total = c + 1; (total & 1u) == 0u; total >>= 1) {
      uint32_t left[8];
      stk.pop(left);
      parent(cv, left, cv, 0u);
    }
    stk.push(cv);
  }
  // the last chunk: per-block length, tail mask, CHUNK_END and (single chunk) ROOT
  const uint32_t c = nch - 1;
  const uint32_t clen = len - (c << 10);
  const uint32_t cblocks = clen == 0 ? 1u : (clen + 63u) >> 6;
  set_iv(cv);
  for (uint32_t b = 0; b < cblocks; b += 2) {
    if (b + 2 < cblocks) lane_line_clamped(q, 8u * c + (b >> 1) + 1u, len, B);
#pragma unroll
    for (uint32_t h = 0; h < 2; ++h) {
      if (h == 1 && b + 1 >= cblocks) break;
      uint32_t m[16];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const uint4 v = A[4 * h + i];
        m[4 * i] = v.x; m[4 * i + 1] = v.y; m[4 * i + 2] = v.z; m[4 * i + 3] = v.w;
      }
      const uint32_t bo = (b + h) << 6;
      const uint32_t blen = clen - bo < 64u ? clen - bo : 64u;  // clen > bo, or both 0
      if (blen < 64u) {
#pragma unroll
        for (int w = 0; w < 16; ++w) {
          const int vb = (int)blen - 4 * w;
          m[w] &= vb >= 4 ? 0xFFFFFFFFu : (vb <= 0 ? 0u : ((1u << (8 * vb)) - 1u));
        }
      }
      const bool end = b + h + 1 == cblocks;
      const uint32_t f = (b + h == 0 ? (uint32_t)CHUNK_START : 0u) | (end ? (uint32_t)CHUNK_END : 0u) |
                         (end && nch == 1 ? (uint32_t)ROOT : 0u);
      compress(cv, m, c, 0u, blen, f);
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) A[i] = B[i];
  }
  while (stk.sp > 0) {
    uint32_t left[8];
    stk.pop(left);
    parent(cv, left, cv, stk.sp == 0 ? (uint32_t)ROOT : 0u);
  }
}

// visiting key: descending chunk count up to MID_CHUNKS, MID_CHUNKS (last) for the rest;
// info[0] += the lane class's chunks, info[1..3] += the 65..256 / 17..64 / <= 16 chunk
// class sizes (wave sums, one atomic each per wave)
extern "C" __global__ void __launch_bounds__(256)
sd_b3_lane_keys(const uint64_t* __restrict__ offs, const uint64_t* __restrict__ lens, uint64_t n,
                uint64_t arena_bytes, int block_key, uint64_t* __restrict__ keys,
                uint32_t* __restrict__ info) {
  __shared__ uint32_t part[4][4];
  uint32_t v[4] = {0u, 0u, 0u, 0u};  // <= 2^24 buffers x 128 chunks: fits u32
  for (uint64_t f = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; f < n;
       f += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t len = lens[f];
    const uint64_t nch = chunks_of(len);
    const bool ok = nch <= MID_CHUNKS && buffer_ok(offs[f], len, arena_bytes);
    if (block_key) {
      const uint64_t blocks = len == 0 ? 1u : (len + 63u) >> 6;  // a 0-byte buffer: one block
      keys[f] = ok ? MID_CHUNKS * 16 - blocks : MID_CHUNKS * 16;
    } else {
      keys[f] = ok ? MID_CHUNKS - nch : MID_CHUNKS;
    }
    v[0] += ok && nch <= LANE_CHUNKS ? (uint32_t)nch : 0u;
    v[1] += ok && nch > SMALL_CHUNKS;
    v[2] += ok && nch > 16 && nch <= SMALL_CHUNKS;
    v[3] += ok && nch <= 16;
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v[k] += __shfl_xor(v[k], d, 64);
  }
  const uint32_t w = threadIdx.x >> 6;
  if ((threadIdx.x & 63u) == 0) {
#pragma unroll
    for (int k = 0; k < 4; ++k) part[w][k] = v[k];
  }
  __syncthreads();
  // one atomic per counter per workgroup over a <= 1,024-workgroup grid (one per wave on
  // the same four words took 0.37 ms for 1 M buffers)
  if (threadIdx.x < 4) {
    const uint32_t k = threadIdx.x;
    const uint32_t sum = part[0][k] + part[1][k] + part[2][k] + part[3][k];
    if (sum) atomicAdd(info + k, sum);
  }
}

extern "C" __global__ void __launch_bounds__(LANE_BLOCK)
sd_b3_batch_lane(const uint8_t* __restrict__ arena, uint64_t arena_bytes,
                 const uint64_t* __restrict__ offs, const uint64_t* __restrict__ lens,
                 const uint32_t* __restrict__ order, uint64_t n, const uint32_t* __restrict__ lane_info,
                 uint32_t* __restrict__ digests) {
  __shared__ uint32_t stack_lds[LANE_LDS_DEPTH][8][LANE_BLOCK];
  const uint64_t t = (uint64_t)blockIdx.x * LANE_BLOCK + threadIdx.x;
  if (t >= n) return;
  const uint32_t f = order[t];
  const uint64_t len = lens[f];
  if (chunks_of(len) > lane_cut(lane_info) || !buffer_ok(offs[f], len, arena_bytes)) return;
  LaneStack stk{stack_lds, threadIdx.x};
  uint32_t cv[8];
  lane_digest(reinterpret_cast<const uint4*>(arena + offs[f]), (uint32_t)len, stk, cv);
#pragma unroll
  for (int k = 0; k < 8; ++k) digests[8ull * f + k] = cv[k];
}

// A large grid (up to 65,536 workgroups: far more than are resident) strides over the work
// list, so the hardware dispatcher balances it at workgroup granularity like K3's one
// workgroup per group; an atomic work cursor over a resident-sized grid ran 14 % slower on
// one 16 GiB buffer (2.41 vs 2.8 TB/s).  4 waves per SIMD like sd_b3_chunk_groups.
extern "C" __global__ void __launch_bounds__(GROUP) __attribute__((amdgpu_waves_per_eu(4)))
sd_b3_batch_groups(const uint8_t* __restrict__ arena, const uint64_t* __restrict__ offs,
                   const uint64_t* __restrict__ lens, const uint32_t* __restrict__ gstart,
                   const uint32_t* __restrict__ groups, const uint32_t* __restrict__ owner,
                   const unsigned long long* __restrict__ gtotal,
                   uint64_t n, uint64_t items_cap, uint32_t* __restrict__ cvs_out,
                   uint32_t* __restrict__ digests, uint32_t* __restrict__ bad) {
  __shared__ uint32_t cvs[GROUP * K3_LANE_CHUNKS][8];
  // the true (u64) total: overlapping buffers can sum past 2^32 groups, where the u32
  // gstart scan wraps and a wrapped total would pass this check
  const uint64_t total = *gtotal;
  if (total > items_cap) {  // lengths beyond arena_bytes: the CV list would overflow
    if (blockIdx.x == 0 && threadIdx.x == 0) atomicOr(bad, 2u);
    return;
  }
  // the item's state is workgroup-uniform: readfirstlane keeps it in SGPRs
  auto uni = [](uint32_t x) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)x); };
  auto uni64 = [&](uint64_t x) { return ((uint64_t)uni((uint32_t)(x >> 32)) << 32) | uni((uint32_t)x); };
  for (uint64_t item = blockIdx.x; item < total; item += gridDim.x) {
    const uint32_t f = uni(owner[item]);
    const uint64_t g = item - uni(gstart[f]);
    const bool single = uni(groups[f]) == 1;
    uint32_t* out8 = single ? digests + 8 * (uint64_t)f : cvs_out + 8 * item;
    group_subtree<K3_LANE_CHUNKS>(arena + uni64(offs[f]), uni64(lens[f]), 0, g, out8,
                                  single ? 1 : 0, cvs);
  }
}

// First reduce level of buffers with > 256 groups, spread over workgroups: workgroup k
// takes the item window [256 k, 256 k + 256) and reduces every 256-CV block of such a
// buffer that STARTS in it (block j of buffer f starts at item gstart[f] + 256 j), writing
// the block's CV over the block's first slot (a 16 GiB buffer: 64 blocks on 64 workgroups
// instead of one workgroup walking all 16,384 CVs, 0.38 ms).
extern "C" __global__ void __launch_bounds__(GROUP)
sd_b3_batch_blocks(const uint32_t* __restrict__ gstart, const uint32_t* __restrict__ groups,
                   const uint32_t* __restrict__ owner, const unsigned long long* __restrict__ gtotal,
                   uint64_t n, uint64_t items_cap, uint32_t* __restrict__ cvs) {
  __shared__ uint32_t work[GROUP][8];
  const uint32_t t = threadIdx.x;
  const uint64_t total = *gtotal;
  if (total > items_cap) return;
  const uint64_t w0 = (uint64_t)blockIdx.x * GROUP;
  if (w0 >= total) return;
  const uint64_t w1 = w0 + GROUP < total ? w0 + GROUP : total;
  const uint32_t f1 = owner[w1 - 1];
  for (uint32_t f = owner[w0]; f <= f1; ++f) {  // buffers with items in the window
    const uint32_t cnt = groups[f];
    if (cnt <= GROUP) continue;
    const uint64_t base = gstart[f];
    for (uint64_t j = w0 > base ? (w0 - base + GROUP - 1) / GROUP : 0;
         base + GROUP * j < w1 && GROUP * j < cnt; ++j) {
      const uint32_t m = (uint32_t)min((uint64_t)GROUP, cnt - GROUP * j);
      uint32_t* blk = cvs + 8 * (base + GROUP * j);
      if (t < m) {
#pragma unroll
        for (int w = 0; w < 8; ++w) work[t][w] = blk[8 * t + w];
      }
      __syncthreads();
      lds_reduce<1>(work, m, false);
      if (t < 8) blk[t] = work[0][t];
      __syncthreads();
    }
  }
}

// Per buffer with >= 2 groups: <= 256 group CVs (or, above 256 groups, the block CVs that
// sd_b3_batch_blocks left at stride 256) pair-and-promote to the ROOT digest in LDS.
extern "C" __global__ void __launch_bounds__(GROUP)
sd_b3_batch_reduce(const uint32_t* __restrict__ gstart, const uint32_t* __restrict__ groups,
                   const unsigned long long* __restrict__ gtotal, uint64_t n, uint64_t items_cap,
                   const uint32_t* __restrict__ cvs_in, uint32_t* __restrict__ digests) {
  __shared__ uint32_t work[GROUP][8];
  __shared__ uint32_t list[GROUP];
  __shared__ uint32_t listed;
  const uint32_t t = threadIdx.x;
  if (*gtotal > items_cap) return;
  // the workgroup scans a window of up to 256 buffers in parallel and lists those with >= 2
  // groups (one buffer per workgroup iteration cost a dependent load per buffer: 0.4 ms for
  // a batch of 1 M small buffers, none of them multi-group); windows of n / grid buffers
  // below that, so a few thousand big buffers still spread over the whole grid
  const uint64_t win = min((uint64_t)GROUP, (n + gridDim.x - 1) / gridDim.x);
  for (uint64_t base = (uint64_t)blockIdx.x * win; base < n; base += (uint64_t)gridDim.x * win) {
    if (t == 0) listed = 0;
    __syncthreads();
    if (t < win && base + t < n && groups[base + t] >= 2) list[atomicAdd(&listed, 1u)] = t;
    __syncthreads();
    const uint32_t k = listed;
    SD_DBG_CHECK(t != 0 || k <= win, "batch reduce: %u buffers listed in a window of %llu", k,
                 (unsigned long long)win);
    for (uint32_t i = 0; i < k; ++i) {
      const uint64_t f = base + list[i];
      const uint32_t cnt = groups[f];
      const uint32_t* in = cvs_in + 8 * (uint64_t)gstart[f];
      // above 256 groups the level-1 block CVs sit at stride 256 (<= 256 of them: 64 GiB)
      const uint32_t stride = cnt <= GROUP ? 1u : GROUP;
      const uint32_t m = cnt <= GROUP ? cnt : (cnt + GROUP - 1) / GROUP;
      if (t < m) {
#pragma unroll
        for (int w = 0; w < 8; ++w) work[t][w] = in[8 * (uint64_t)t * stride + w];
      }
      __syncthreads();
      lds_reduce<1>(work, m, true);
      if (t < 8) digests[8 * f + t] = work[0][t];
      __syncthreads();
    }
    __syncthreads();  // `listed` and `list` read by every wave before the next trip resets them
  }
}

// one buffer at offset 0 (sd_cas_checksum_dev): its offs/lens words and the flag, in one
// tiny kernel rather than three runtime fills
extern "C" __global__ void sd_b3_single_setup(uint64_t* __restrict__ ol, uint64_t len,
                                              uint32_t* __restrict__ bad) {
  if (threadIdx.x == 0) { ol[0] = 0; ol[1] = len; *bad = 0; }
}

hipError_t checksum_single_setup(uint64_t* d_ol, uint64_t len, uint32_t* d_bad, hipStream_t s) {
  sd_b3_single_setup<<<1, 64, 0, s>>>(d_ol, len, d_bad);
  return hipGetLastError();
}

static inline size_t al256c(size_t x) { return (x + 255) / 256 * 256; }

SD_DBG_ACCESSOR(sd_dbg_violations_checksum)

// work items of the big-buffer list: <= n + arena_bytes / 1 MiB (disjoint buffers)
static inline uint64_t batch_items_cap(uint64_t n, uint64_t arena_bytes) {
  return n + arena_bytes / (GROUP_CHUNKS * 1024) + 1;
}

static inline bool lane_path(uint64_t n) { return n >= LANE_MIN_BUFFERS; }

size_t checksum_batch_workspace_bytes(uint64_t n, uint64_t arena_bytes) {
  // groups | gstart | scan partials | group total (u64) | owner | cvs
  //   [| lane class total | lane keys | sorted keys | order | sort ws]
  const uint64_t items = batch_items_cap(n, arena_bytes);
  size_t b = 2 * al256c((n + 1) * 4) + al256c((n / 4096 + 2) * 4) + 256 + al256c(items * 4) +
             al256c(items * 32);
  if (lane_path(n)) b += 256 + 2 * al256c(n * 8) + al256c(n * 4) + sort_workspace_bytes(n);
  return b + 256;
}

hipError_t checksum_batch_device(const uint8_t* arena, uint64_t arena_bytes, const uint64_t* offs,
                                 const uint64_t* lens, uint64_t n, uint32_t* d_digests,
                                 uint32_t* d_bad, void* ws, hipStream_t s) {
  if (n == 0) return hipSuccess;
  if (n > (1ull << 24)) return hipErrorInvalidValue;  // the u32 scan: <= 4096^2 buffers
  const uint64_t items = batch_items_cap(n, arena_bytes);
  // item indices (owner, gstart) are u32: an arena past 4 PiB is refused
  if (items > 0xFFFFFFFFull) return hipErrorInvalidValue;
  char* p = (char*)ws;
  uint32_t* groups = (uint32_t*)p; p += al256c((n + 1) * 4);
  uint32_t* gstart = (uint32_t*)p; p += al256c((n + 1) * 4);
  uint32_t* partial = (uint32_t*)p; p += al256c((n / 4096 + 2) * 4);
  unsigned long long* gtotal = (unsigned long long*)p; p += 256;
  uint32_t* owner = (uint32_t*)p; p += al256c(items * 4);
  uint32_t* cvs = (uint32_t*)p; p += al256c(items * 32);
  const bool lane = lane_path(n);
  uint32_t* lane_info = nullptr;  // LaneInfo counters (zeroed by the count kernel)
  uint32_t* order = nullptr;
  if (lane) { lane_info = (uint32_t*)p; p += 256; }
  const uint32_t nb = (uint32_t)((n + 255) / 256);
  sd_b3_batch_count<<<nb, 256, 0, s>>>(offs, lens, n, arena_bytes, groups, d_bad, lane_info);
  hipError_t e = exclusive_scan_u32(groups, gstart, n, partial, s, gtotal);
  if (e != hipSuccess) return e;
  sd_b3_batch_owner<<<(uint32_t)std::min<uint64_t>((items + 255) / 256, 2048), 256, 0, s>>>(
      gstart, gtotal, n, items, owner);
  if (lane) {
    // buffers of <= lane_cut() chunks one per lane, by descending chunk count
    uint64_t* lkeys = (uint64_t*)p; p += al256c(n * 8);
    uint64_t* skeys = (uint64_t*)p; p += al256c(n * 8);
    order = (uint32_t*)p; p += al256c(n * 4);
    const bool block_key = arena_bytes <= n * LANE_BLOCK_KEY_MEAN;
    sd_b3_lane_keys<<<std::min<uint32_t>(nb, 1024), 256, 0, s>>>(offs, lens, n, arena_bytes,
                                                               block_key ? 1 : 0, lkeys, lane_info);
    e = radix_sort_pairs(lkeys, nullptr, skeys, order, n, 0,
                         block_key ? LANE_KEY_BITS_BLOCKS : LANE_KEY_BITS_CHUNKS, p, s);
    if (e != hipSuccess) return e;
    sd_b3_batch_lane<<<(uint32_t)((n + LANE_BLOCK - 1) / LANE_BLOCK), LANE_BLOCK, LANE_LDS_PAD, s>>>(
        arena, arena_bytes, offs, lens, order, n, lane_info, d_digests);
  }
  // small buffers (those the lane kernel does not take): <= 16 chunks four per wave, 17..64
  // chunks one per wave (up to 8 workgroups of 4 waves per CU); then 65..256 chunks
  sd_b3_batch_small16<<<(uint32_t)std::min<uint64_t>((n + 15) / 16, 256 * 8), 256, 0, s>>>(
      arena, arena_bytes, offs, lens, n, order, lane_info, d_digests);
  sd_b3_batch_small64<<<(uint32_t)std::min<uint64_t>((n + 3) / 4, 256 * 8), 256, 0, s>>>(
      arena, arena_bytes, offs, lens, n, order, lane_info, d_digests);
  sd_b3_batch_mid<<<(uint32_t)std::min<uint64_t>((n + 3) / 4, 256 * 8), 256, 0, s>>>(
      arena, arena_bytes, offs, lens, n, order, lane_info, d_digests);
  // big buffers: a grid of up to 65,536 workgroups strides over the item list (those past
  // the list's end exit at once)
  sd_b3_batch_groups<<<(uint32_t)std::min<uint64_t>(items, 65536), GROUP, 0, s>>>(
      arena, offs, lens, gstart, groups, owner, gtotal, n, items, cvs, d_digests, d_bad);
  sd_b3_batch_blocks<<<(uint32_t)((items + GROUP - 1) / GROUP), GROUP, 0, s>>>(
      gstart, groups, owner, gtotal, n, items, cvs);
  sd_b3_batch_reduce<<<(uint32_t)std::min<uint64_t>(n, 256 * 4), GROUP, 0, s>>>(
      gstart, groups, gtotal, n, items, cvs, d_digests);
  return hipGetLastError();
}

size_t checksum_workspace_bytes(uint64_t len) {
  const uint64_t nchunks = len == 0 ? 1 : (len + 1023) >> 10;
  const uint64_t g = (nchunks + GROUP_CHUNKS - 1) / GROUP_CHUNKS;
  return 2 * ((g * 32 + 255) / 256 * 256) + 512;
}

// Reduce `cnt` CVs at d_cvs (ping-pong with `tmp`) to one; result in *result (device).
static hipError_t reduce_to_one(uint32_t* a, uint32_t* b, uint64_t cnt, bool root,
                                uint32_t** result, hipStream_t s) {
  while (cnt > 1) {
    const uint64_t g = (cnt + GROUP - 1) / GROUP;
    sd_b3_reduce_cvs<<<(uint32_t)g, GROUP, 0, s>>>(a, cnt, b, root ? 1 : 0);
    uint32_t* t = a; a = b; b = t;
    cnt = g;
  }
  *result = a;
  return hipGetLastError();
}

hipError_t checksum_device(const uint8_t* data, uint64_t len, uint64_t chunk0, bool root,
                           uint32_t* d_out8, void* ws, hipStream_t s) {
  const uint64_t nchunks = len == 0 ? 1 : (len + 1023) >> 10;
  const uint64_t g = (nchunks + GROUP_CHUNKS - 1) / GROUP_CHUNKS;
  if (g >= (1ull << 31)) return hipErrorInvalidValue;
  uint32_t* a = (uint32_t*)ws;
  uint32_t* b = (uint32_t*)((char*)ws + (g * 32 + 255) / 256 * 256);
  sd_b3_chunk_groups<<<(uint32_t)g, GROUP, 0, s>>>(data, len, chunk0, a, root ? 1 : 0);
  uint32_t* res;
  hipError_t e = reduce_to_one(a, b, g, root, &res, s);
  if (e != hipSuccess) return e;
  return hipMemcpyAsync(d_out8, res, 32, hipMemcpyDeviceToDevice, s);
}

hipError_t reduce_cvs_device(const uint32_t* d_cvs, uint64_t cnt, uint32_t* d_out8, void* ws,
                             hipStream_t s) {
  if (cnt == 0) return hipErrorInvalidValue;
  const uint64_t g = (cnt + GROUP - 1) / GROUP;
  uint32_t* a = (uint32_t*)ws;
  uint32_t* b = (uint32_t*)((char*)ws + (g * 32 + 255) / 256 * 256);
  if (cnt == 1) return hipMemcpyAsync(d_out8, d_cvs, 32, hipMemcpyDeviceToDevice, s);
  sd_b3_reduce_cvs<<<(uint32_t)g, GROUP, 0, s>>>(d_cvs, cnt, a, 1);
  uint32_t* res;
  hipError_t e = reduce_to_one(a, b, g, true, &res, s);
  if (e != hipSuccess) return e;
  return hipMemcpyAsync(d_out8, res, 32, hipMemcpyDeviceToDevice, s);
}

}  // namespace sdcas
