// cas_hash.hip — batched generate_cas_id on gfx950 (K1 sampled path, K2 whole-file path).
//
// Replaces, per batch, the per-file hashing of core/src/object/cas.rs:23-62:
//   message M(s) = le64(size) || content, content = whole file (size <= 102,400,
//   cas.rs:27-29) or header 8 KiB || 4 x 10 KiB samples || footer 8 KiB (cas.rs:31-58,
//   gathered on the host); cas_id = hex(BLAKE3(M)[0..8]) (cas.rs:61).
//
// Mapping: ONE FILE PER LANE.  Every lane walks its own message and keeps the BLAKE3
// chaining-value stack in an LDS column of its own.  For the sampled path every file has
// the same 57 chunks, so all control flow (block loop, stack merges) is wave-uniform and
// every lane does useful work in every instruction: 953 compressions per lane, no
// cross-lane traffic.  For the whole-file path files are pre-sorted by message length
// (on-device key sort) so the lanes of a wave finish together.
//
// Memory: each lane streams its message in 128-B lines (a block pair, 8 x
// global_load_dwordx4), two lines per loop iteration.  The le64(size) prefix
// shifts the content by exactly two 32-bit words, which becomes register renaming (a
// 2-word carry), not byte shuffling.
//
// Bound: VALU issue.  On gfx950 v_alignbit_b32 / v_add3_u32 (like every 3-input or SDWA
// VALU op except v_bitop3) issue at half rate (tools/ubench_valu.hip,
// profiles/r01_ubench_valu.log), so a compression costs ~1014 full-rate issue slots.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "blake3_device.hpp"
#include "sd_kernels.h"
#include "sd_mix.h"

namespace sdcas {

// ---- K1: the sampled path, specialised --------------------------------------------
// Every message is le64(size) || 57,344 B: 56 full chunks (448 block PAIRS) + one 8-byte
// tail chunk.  A lane fetches one whole 128-B line (a block pair, 8 x dwordx4 issued back
// to back) per batch, so each line is consumed while it is still in L2 (fetching 64 B per
// block let the other half be evicted between blocks and doubled the HBM traffic), and
// both lines of an iteration are in flight together (16 x dwordx4); the other waves of the
// SIMD cover their latency.

constexpr uint32_t SAMPLED_PAIRS = SAMPLED_CONTENT_LEN / 128;  // 448
constexpr uint32_t SAMPLED_CHUNKS = SAMPLED_CONTENT_LEN / 1024;  // 56 full chunks
static_assert(SAMPLED_PAIRS == 8 * SAMPLED_CHUNKS, "the sampled content is whole chunks of 8 lines");

// One 128-B line (block pair P) of the lane's content: 8 x dwordx4 issued back to back.
// (The A/B variants — non-temporal loads, 1.6x slower; 64-file tiled LINE / QUAD layouts —
// live in tools/ubench_k1.hip with their measurements.)
__device__ __forceinline__ void load_pair(const uint4* __restrict__ q, uint32_t P, uint4 (&buf)[8]) {
  const uint4* p = q + 8u * P;
#pragma unroll
  for (int i = 0; i < 8; ++i) buf[i] = p[i];
}

// Compress message blocks 2P and 2P+1 of chunk `ctr` from the line in A; the 2-word
// carry is the tail of the previous line (the 8-byte size prefix shift).
__device__ __forceinline__ void compress_pair(uint32_t (&cv)[8], const uint4 (&A)[8],
                                              uint32_t& c0, uint32_t& c1, uint32_t ctr,
                                              uint32_t f0, uint32_t f1) {
  {
    const uint32_t m[16] = {c0, c1, A[0].x, A[0].y, A[0].z, A[0].w, A[1].x, A[1].y,
                            A[1].z, A[1].w, A[2].x, A[2].y, A[2].z, A[2].w, A[3].x, A[3].y};
    compress(cv, m, ctr, 0u, BLOCK_LEN, f0);
  }
  {
    const uint32_t m[16] = {A[3].z, A[3].w, A[4].x, A[4].y, A[4].z, A[4].w, A[5].x, A[5].y,
                            A[5].z, A[5].w, A[6].x, A[6].y, A[6].z, A[6].w, A[7].x, A[7].y};
    compress(cv, m, ctr, 0u, BLOCK_LEN, f1);
  }
  c0 = A[7].z;
  c1 = A[7].w;
}

// The 5-deep chaining-value stack lives in LDS, word-major [depth][word][thread] so every
// push/pop is a conflict-free dword access.  It is touched once per 1 KiB chunk (16
// compressions), and moving its 40 words per lane out of VGPRs takes the kernel from 3
// to 4 waves per SIMD (VGPR budget <= 128); 80 KiB per 512-lane block = 2 blocks/CU.
constexpr int SAMPLED_DEPTH = 5;  // popcount(55) pending subtrees at most
constexpr int SAMPLED_BLOCK = 512;  // 256: 1-2 % slower, 128: 4 % (profiles/r01_k1_block_ab.log)

template <int B = SAMPLED_BLOCK>
struct LdsStack {
  uint32_t (*s)[8][B];
  uint32_t t;
  uint32_t sp = 0;  // wave-uniform on the sampled path
  __device__ __forceinline__ void push(const uint32_t (&cv)[8]) {
#pragma unroll
    for (int w = 0; w < 8; ++w) s[sp][w][t] = cv[w];
    ++sp;
  }
  __device__ __forceinline__ void pop(uint32_t (&out)[8]) {
    --sp;
#pragma unroll
    for (int w = 0; w < 8; ++w) out[w] = s[sp][w][t];
  }
};

template <int BLK = SAMPLED_BLOCK>
__device__ __forceinline__ uint64_t cas_lane_sampled(const uint4* __restrict__ q, uint64_t size,
                                                     LdsStack<BLK>& stk) {
  uint32_t c0 = (uint32_t)size, c1 = (uint32_t)(size >> 32);
  uint4 A[8], B[8];
  uint32_t cv[8];
  for (uint32_t c = 0; c < SAMPLED_CHUNKS; ++c) {
    set_iv(cv);
#pragma unroll 1
    for (uint32_t pp = 0; pp < 4; ++pp) {  // 4 x (pair A, pair B) = 16 blocks
      // both lines at the iteration start: a pair prefetched across the back edge was
      // renamed and copied back (32 v_mov_b64 per iteration, 687.5 VALU instructions per
      // compression); the load latency is covered by the SIMD's other three waves
      // (681.5 per compression, +0.3-0.5 %: profiles/r05/ab_k1_prefetch/)
      const uint32_t P = 8u * c + 2u * pp;
      load_pair(q, P, A);
      load_pair(q, P + 1, B);
      compress_pair(cv, A, c0, c1, c, pp == 0 ? (uint32_t)CHUNK_START : 0u, 0u);
      compress_pair(cv, B, c0, c1, c, 0u, pp == 3 ? (uint32_t)CHUNK_END : 0u);
    }
    // left-balanced tree: merge while the completed-chunk count has trailing zeros
    uint32_t total = c + 1;
    while ((total & 1u) == 0u) {
      uint32_t left[8];
      stk.pop(left);
      parent(cv, left, cv, 0u);
      total >>= 1;
    }
    stk.push(cv);
  }
  // tail chunk 56: the last 8 content bytes (the carry), one 8-byte block
  {
    const uint32_t m[16] = {c0, c1, 0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u};
    set_iv(cv);
    compress(cv, m, SAMPLED_CHUNKS, 0u, 8u, CHUNK_START | CHUNK_END);
  }
  // 56 = 0b111000: the stack holds the 32-, 16- and 8-chunk subtrees
#pragma unroll
  for (int d = 0; d < 3; ++d) {
    uint32_t left[8];
    stk.pop(left);
    parent(cv, left, cv, d == 2 ? (uint32_t)ROOT : 0u);
  }
  return key_of(cv);
}

// K1: sampled path, uniform 57,344-B contents at a fixed stride (>= 57,344, 16-B aligned).
// Two grid shapes of the same lane program: 512-lane workgroups (80 KiB of LDS stack, 2 per
// CU) for batches of >= 2 quanta, and 256-lane workgroups (40 KiB, 4 per CU) below: a batch
// of one quantum is 128 workgroups of 512 lanes, which the dispatcher puts on 128 CUs at 2
// waves per SIMD — half the chip idle and twice the latency (measured 2.27 vs 1.15 ms for
// 65,536 files, profiles/r02_latency_sweep.log) — while 256 workgroups of 256 lanes put one
// wave on every SIMD.
template <int B>
__device__ __forceinline__ void sampled_kernel_body(const uint8_t* __restrict__ content,
                                                    uint64_t stride,
                                                    const uint64_t* __restrict__ sizes, uint64_t n,
                                                    uint64_t* __restrict__ keys) {
  __shared__ uint32_t stack_lds[SAMPLED_DEPTH][8][B];
  const uint64_t f = (uint64_t)blockIdx.x * B + threadIdx.x;
  if (f >= n) return;  // no barrier below: each lane only touches its own stack column
  LdsStack<B> stk{stack_lds, threadIdx.x};
  const uint4* q = reinterpret_cast<const uint4*>(content + f * stride);
  keys[f] = cas_lane_sampled<B>(q, sizes[f], stk);
}

extern "C" __global__ void __launch_bounds__(SAMPLED_BLOCK)
sd_cas_sampled_kernel(const uint8_t* __restrict__ content, uint64_t stride,
                      const uint64_t* __restrict__ sizes, uint64_t n,
                      uint64_t* __restrict__ keys) {
  sampled_kernel_body<SAMPLED_BLOCK>(content, stride, sizes, n, keys);
}

constexpr int SAMPLED_BLOCK_NARROW = 256;
extern "C" __global__ void __launch_bounds__(SAMPLED_BLOCK_NARROW)
sd_cas_sampled_kernel_256(const uint8_t* __restrict__ content, uint64_t stride,
                          const uint64_t* __restrict__ sizes, uint64_t n,
                          uint64_t* __restrict__ keys) {
  sampled_kernel_body<SAMPLED_BLOCK_NARROW>(content, stride, sizes, n, keys);
}

// ---- K1G: K1 + the grouping's partition, fused (sd_cas_hash_group_sampled_dev) ----------
// The Object grouping needs each key once more after K1 has written it: the standalone chain
// reads the keys back (bucket totals, 8 B/key), prefills rep (4 B/key), then scatters the
// keys into coarse-bucket order (8 B read + 12 B write) before the bucket tables.  K1 holds
// every key in a register when it finishes, so K1G does that partition in its epilogue
// instead: the lane's (mixed key, file) row goes straight into a FIXED-capacity region of
// its coarse bucket (the top 8 bits of mix64(key)); the workgroup ranks its lanes per bucket
// in LDS (the CV stack's LDS, dead by then) and reserves each bucket's run with one device
// atomic.  The chain after K1G is one bucket-table launch.  Regions are sized mean + 8
// sigma + 64 rows for uniform keys; a bucket that outgrows its region (heavily duplicated
// content: every copy of a file lands in one bucket) keeps counting in its cursor, appends
// its extra rows to the set's spill list (one reservation per workgroup that has any) and
// sets *overflow; that region's table workgroup reads its region rows and its spilled rows
// (sd_bucket_min_regions) — only the overflowed regions pay, on the device, no host regroup.
struct RegionOut {
  uint64_t* rkeys;     // [REGIONS][cap] mixed keys
  uint32_t* rfile;     // [REGIONS][cap] file index
  uint32_t* cursor;    // [REGION_SET_WORDS] rows reserved per region, then the spill count and
                       // the full-region count at REGION_SPILL_WORD; zero on entry (the bucket
                       // tables re-zero them)
  uint64_t cap;
  uint64_t* spill_keys;   // rows past their region's capacity (mixed key, file), unordered
  uint32_t* spill_file;
  uint32_t* rep;       // rep[f] = f: the bucket tables store only where a key's minimum differs
  uint32_t* overflow;  // set when a region is full
  // objects[0]: zeroed here, the bucket tables add the distinct keys; objects[1]: zeroed
  // here, the tables' carve cursor for the global tables of overflowed regions
  unsigned long long* objects;
};

template <int B>
__device__ __forceinline__ void sampled_group_kernel_body(const uint8_t* __restrict__ content,
                                                          uint64_t stride,
                                                          const uint64_t* __restrict__ sizes,
                                                          uint64_t n, uint64_t* __restrict__ keys,
                                                          RegionOut ro) {
  __shared__ uint32_t stack_lds[SAMPLED_DEPTH][8][B];
  const uint64_t f = (uint64_t)blockIdx.x * B + threadIdx.x;
  const bool live = f < n;
  uint64_t key = 0;
  if (live) {  // exactly K1's lane program
    LdsStack<B> stk{stack_lds, threadIdx.x};
    const uint4* q = reinterpret_cast<const uint4*>(content + f * stride);
    key = cas_lane_sampled<B>(q, sizes[f], stk);
    keys[f] = key;
    ro.rep[f] = (uint32_t)f;
  }
  if (blockIdx.x == 0 && threadIdx.x < 2) ro.objects[threadIdx.x] = 0;
  // epilogue: the stack columns are dead once every lane has its root
  // REGIONS counters, REGIONS run bases, REGIONS spill offsets, the spill total and base
  uint32_t* hist = &stack_lds[0][0][0];
  uint32_t* base = hist + REGIONS;
  uint32_t* spoff = base + REGIONS;
  uint32_t* sp = spoff + REGIONS;  // sp[0] = this workgroup's spilled rows, sp[1] = their base
  static_assert(3 * REGIONS + 2 <= SAMPLED_DEPTH * 8 * B, "the epilogue fits the stack LDS");
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < REGIONS; i += B) hist[i] = 0;
  if (threadIdx.x == 0) sp[0] = 0;
  __syncthreads();
  const uint64_t m = mix64(key);
  const uint32_t bkt = (uint32_t)(m >> (64 - REGION_BITS));
  const uint32_t r = live ? atomicAdd(&hist[bkt], 1u) : 0u;
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < REGIONS; i += B) {
    const uint32_t h = hist[i];
    const uint32_t g = h ? atomicAdd(&ro.cursor[i], h) : 0u;
    base[i] = g;
    // rows past the region's capacity: this workgroup's run of them for region i
    const uint64_t lo = g > ro.cap ? g : ro.cap;
    const uint32_t over = g + h > lo ? (uint32_t)(g + h - lo) : 0u;
    spoff[i] = over ? atomicAdd(&sp[0], over) : 0u;
    if (g <= ro.cap && g + h > ro.cap) atomicAdd(&ro.cursor[REGION_SPILL_WORD + 1], 1u);  // it filled
  }
  __syncthreads();
  if (sp[0]) {  // (uniform) a region is full: one spill reservation for the workgroup
    if (threadIdx.x == 0) {
      sp[1] = atomicAdd(&ro.cursor[REGION_SPILL_WORD], sp[0]);
      atomicOr(ro.overflow, 1u);
    }
    __syncthreads();
  }
  if (live) {
    const uint64_t slot = (uint64_t)base[bkt] + r;
    if (slot < ro.cap) {
      ro.rkeys[(uint64_t)bkt * ro.cap + slot] = m;
      ro.rfile[(uint64_t)bkt * ro.cap + slot] = (uint32_t)f;
    } else {
      const uint64_t d = (uint64_t)sp[1] + spoff[bkt] + (slot - (base[bkt] > ro.cap ? base[bkt] : ro.cap));
      ro.spill_keys[d] = m;
      ro.spill_file[d] = (uint32_t)f;
    }
  }
}

extern "C" __global__ void __launch_bounds__(SAMPLED_BLOCK)
sd_cas_sampled_group_kernel(const uint8_t* __restrict__ content, uint64_t stride,
                            const uint64_t* __restrict__ sizes, uint64_t n,
                            uint64_t* __restrict__ keys, RegionOut ro) {
  sampled_group_kernel_body<SAMPLED_BLOCK>(content, stride, sizes, n, keys, ro);
}

extern "C" __global__ void __launch_bounds__(SAMPLED_BLOCK_NARROW)
sd_cas_sampled_group_kernel_256(const uint8_t* __restrict__ content, uint64_t stride,
                                const uint64_t* __restrict__ sizes, uint64_t n,
                                uint64_t* __restrict__ keys, RegionOut ro) {
  sampled_group_kernel_body<SAMPLED_BLOCK_NARROW>(content, stride, sizes, n, keys, ro);
}

// ---- K2: the whole-file (packed) path ------------------------------------------------
// Ragged messages of up to PACKED_MAX_CHUNKS chunks, one file per lane, lanes visited
// longest-first (on-device length sort) so a wave's lanes run the same trip counts.
// Same line-batched loads as K1 (a 128-B block pair per batch, prefetched one pair
// ahead; quads past the content are not loaded, bytes past the message are masked) and
// an LDS CV stack (per-lane depth, word-major).
// popcount(c) <= 6 pending subtrees for c <= 103 completed chunks: the bottom one (the
// largest subtree) stays in VGPRs and the other 5 live in LDS, 160 B per lane = 40 KiB per
// 256-lane block, so 4 blocks fill a CU's 160 KiB and K2 runs 4 waves per SIMD (a 6-deep
// LDS stack, 48 KiB per block, held it to 3).
constexpr int PACKED_DEPTH = 6;
constexpr int PACKED_LDS_DEPTH = PACKED_DEPTH - 1;
constexpr int PACKED_BLOCK = 256;

struct PackedStack {
  uint32_t (*s)[8][PACKED_BLOCK];
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

// Always 8 x 16-B loads: a quad past the content is re-pointed at quad 0 (in bounds; an
// empty content still has 16 readable bytes, see the ABI) instead of being predicated off
// — a `cond ? q[i] : 0` load is lowered to four dword loads per quad.  Its garbage can
// only reach the message's final block, which mask_tail() zeroes past the end.
__device__ __forceinline__ void load_pair_pred(const uint4* __restrict__ q, uint32_t P,
                                               uint32_t clen, uint4 (&buf)[8]) {
  const uint32_t b0 = P << 7;
#pragma unroll
  for (int i = 0; i < 8; ++i) buf[i] = q[(b0 + 16u * i < clen) ? 8u * P + i : 0u];
}

__device__ __forceinline__ void mask_tail(uint32_t (&m)[16], uint32_t blen) {
#pragma unroll
  for (int w = 0; w < 16; ++w) {
    const int vb = (int)blen - 4 * w;
    m[w] &= vb >= 4 ? 0xFFFFFFFFu : (vb <= 0 ? 0u : ((1u << (8 * vb)) - 1u));
  }
}

// One FULL 1 KiB chunk (not the message's last) of a K2 lane: 16 blocks of 64 B with the
// chunk flags on blocks 0 and 15 — none of the generic loop's per-block length, mask and
// flag logic, and unclamped loads for the chunk's own pairs (a full chunk's content quads
// are readable: clen > 1024c + 1016 puts its 16-B round-up past the chunk).  Only the
// prefetch of the next chunk's first pair is clamped.  A holds pair 8c on entry and pair
// 8(c+1) on exit.  Lanes of a wave share the chunk count (the visiting order is sorted on
// it), so this loop is wave-uniform.
__device__ __forceinline__ void packed_full_chunk(const uint4* __restrict__ q, uint32_t clen,
                                                  uint32_t c, uint32_t (&cv)[8], uint4 (&A)[8],
                                                  uint4 (&B)[8], uint32_t& c0, uint32_t& c1) {
  set_iv(cv);
  // K1's ping-pong schedule (no register moves): pairs 0..5 in the loop, 6 and 7 peeled so
  // that the clamped prefetch of the next chunk's first pair does not merge with the
  // unclamped loads into per-dword select loads (that merge measured 2.8x slower)
#pragma unroll 1
  for (uint32_t pp = 0; pp < 3; ++pp) {
    const uint32_t P = 8u * c + 2u * pp;
    load_pair(q, P + 1, B);
    compress_pair(cv, A, c0, c1, c, pp == 0 ? (uint32_t)CHUNK_START : 0u, 0u);
    load_pair(q, P + 2, A);
    compress_pair(cv, B, c0, c1, c, 0u, 0u);
  }
  load_pair(q, 8u * c + 7u, B);
  compress_pair(cv, A, c0, c1, c, 0u, 0u);
  load_pair_pred(q, 8u * c + 8u, clen, A);
  compress_pair(cv, B, c0, c1, c, 0u, CHUNK_END);
}

__device__ __forceinline__ uint64_t cas_lane_packed(const uint4* __restrict__ q, uint32_t clen,
                                                    uint64_t size,
                                                    PackedStack& stk) {
  const uint32_t mlen = clen + 8u;
  const uint32_t nblocks = (mlen + 63u) >> 6;   // >= 1
  const uint32_t nchunks = (mlen + 1023u) >> 10;
  const uint32_t npairs = (nblocks + 1u) >> 1;
  uint32_t c0 = (uint32_t)size, c1 = (uint32_t)(size >> 32);
  uint4 A[8], B[8];
  load_pair_pred(q, 0, clen, A);
  uint32_t cv[8];
  for (uint32_t c = 0; c + 1 < nchunks; ++c) {
    packed_full_chunk(q, clen, c, cv, A, B, c0, c1);
    uint32_t total = c + 1;
    while ((total & 1u) == 0u) {
      uint32_t left[8];
      stk.pop(left);
      parent(cv, left, cv, 0u);
      total >>= 1;
    }
    stk.push(cv);
  }
  {
    // the message's last chunk: generic blocks with length, tail mask and ROOT flags
    const uint32_t c = nchunks - 1;
    const uint32_t cblocks = nblocks - 16u * c;
    set_iv(cv);
    for (uint32_t b = 0; b < cblocks; b += 2) {
      const uint32_t P = 8u * c + (b >> 1);
      if (P + 1 < npairs) load_pair_pred(q, P + 1, clen, B);
      const uint32_t j = 16u * c + b;  // global block index of the pair's first block
      const bool root1 = c == 0;
      {
        uint32_t m[16] = {c0, c1, A[0].x, A[0].y, A[0].z, A[0].w, A[1].x, A[1].y,
                          A[1].z, A[1].w, A[2].x, A[2].y, A[2].z, A[2].w, A[3].x, A[3].y};
        const uint32_t rem = mlen - (j << 6), blen = rem < 64u ? rem : 64u;
        if (blen < 64u) mask_tail(m, blen);
        const bool end = (b + 1 == cblocks);
        const uint32_t f = (b == 0 ? (uint32_t)CHUNK_START : 0u) | (end ? (uint32_t)CHUNK_END : 0u) |
                           (end && root1 ? (uint32_t)ROOT : 0u);
        compress(cv, m, c, 0u, blen, f);
      }
      if (b + 1 < cblocks) {
        uint32_t m[16] = {A[3].z, A[3].w, A[4].x, A[4].y, A[4].z, A[4].w, A[5].x, A[5].y,
                          A[5].z, A[5].w, A[6].x, A[6].y, A[6].z, A[6].w, A[7].x, A[7].y};
        const uint32_t rem = mlen - ((j + 1) << 6), blen = rem < 64u ? rem : 64u;
        if (blen < 64u) mask_tail(m, blen);
        const bool end = (b + 2 == cblocks);
        const uint32_t f = (end ? (uint32_t)CHUNK_END : 0u) | (end && root1 ? (uint32_t)ROOT : 0u);
        compress(cv, m, c, 0u, blen, f);
      }
      c0 = A[7].z;
      c1 = A[7].w;
#pragma unroll
      for (int i = 0; i < 8; ++i) A[i] = B[i];
    }
  }
  while (stk.sp > 0) {
    uint32_t left[8];
    stk.pop(left);
    parent(cv, left, cv, stk.sp == 0 ? (uint32_t)ROOT : 0u);
  }
  return key_of(cv);
}

// ---- K1L: chunk-parallel latency path (small batches) ---------------------------------
// A file per wave (a lane per 1 KiB chunk) or per 16-lane segment (4+ chunks per lane),
// then a level-wise pair-and-promote merge of the lanes' subtree CVs across lanes (DPP row
// shifts inside a 16-lane row).  A file's latency is ~16 + log2(chunks) compression times
// instead of the lane-per-file kernels' 953, at ~68 % (wave per file) / ~84 % (4 files per
// wave) lane efficiency — the right trade when a batch is too small to fill the chip (the
// reference's job step is 100 files, file_identifier/mod.rs:34).  Chosen by the host below
// sd_cas_set_latency_threshold; the shape by sd_cas_set_chunkpar_split.
constexpr int CP_MAX_CHUNKS = 104;

// CV of chunk c of M = le64(size) || content[0, clen); ROOT when M is a single chunk.
__device__ __forceinline__ void cas_chunk_cv(const uint4* __restrict__ q, uint32_t clen,
                                             uint64_t size, uint32_t c, uint32_t (&cv)[8]) {
  const uint32_t mlen = clen + 8u;
  const uint32_t nblocks = (mlen + 63u) >> 6;
  const uint32_t nchunks = (mlen + 1023u) >> 10;
  const bool last = (c + 1 == nchunks);
  const bool root = last && c == 0;
  const uint32_t cblocks = last ? (nblocks - 16u * c) : 16u;
  // message words [256c, 256c+2) = content words [256c-2, 256c): the size for chunk 0
  uint32_t c0 = (uint32_t)size, c1 = (uint32_t)(size >> 32);
  if (c > 0) {
    const uint4 p = q[(64u * c - 1u) * 16u < clen ? 64u * c - 1u : 0u];
    c0 = p.z;
    c1 = p.w;
  }
  uint4 A[8], B[8];
  load_pair_pred(q, 8u * c, clen, A);
  set_iv(cv);
  for (uint32_t b = 0; b < cblocks; b += 2) {
    const uint32_t P = 8u * c + (b >> 1);
    if (b + 2 < cblocks) load_pair_pred(q, P + 1, clen, B);
    const uint32_t j = 16u * c + b;
    {
      uint32_t m[16] = {c0, c1, A[0].x, A[0].y, A[0].z, A[0].w, A[1].x, A[1].y,
                        A[1].z, A[1].w, A[2].x, A[2].y, A[2].z, A[2].w, A[3].x, A[3].y};
      const uint32_t rem = mlen - (j << 6), blen = rem < 64u ? rem : 64u;
      if (blen < 64u) mask_tail(m, blen);
      const bool end = (b + 1 == cblocks);
      const uint32_t f = (b == 0 ? (uint32_t)CHUNK_START : 0u) | (end ? (uint32_t)CHUNK_END : 0u) |
                         (end && root ? (uint32_t)ROOT : 0u);
      compress(cv, m, c, 0u, blen, f);
    }
    if (b + 1 < cblocks) {
      uint32_t m[16] = {A[3].z, A[3].w, A[4].x, A[4].y, A[4].z, A[4].w, A[5].x, A[5].y,
                        A[5].z, A[5].w, A[6].x, A[6].y, A[6].z, A[6].w, A[7].x, A[7].y};
      const uint32_t rem = mlen - ((j + 1) << 6), blen = rem < 64u ? rem : 64u;
      if (blen < 64u) mask_tail(m, blen);
      const bool end = (b + 2 == cblocks);
      const uint32_t f = (end ? (uint32_t)CHUNK_END : 0u) | (end && root ? (uint32_t)ROOT : 0u);
      compress(cv, m, c, 0u, blen, f);
    }
    c0 = A[7].z;
    c1 = A[7].w;
#pragma unroll
    for (int i = 0; i < 8; ++i) A[i] = B[i];
  }
}

// Value of `x` held by lane (lane + S) of the same file segment (S < SEG, a power of two;
// lanes past the wave's end read 0 and are never used).  S < 16 stays inside a DPP row:
// DPP row_shl:S (lane i reads lane i + S of its 16-lane row) — no LDS, no extra issue.
// S = 16, 32 (only in 64-lane segments) cross rows: ds_bpermute (__shfl_down).
template <uint32_t S>
__device__ __forceinline__ uint32_t from_lane_above(uint32_t x) {
  if constexpr (S < 16)
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x100 | (int)S, 0xF, 0xF, true);
  else
    return __shfl_down(x, S, 64);
}

// Level-wise pair-and-promote across the lanes of a segment: item i (a subtree CV) sits in
// segment lane i*s at the level with stride s; the left lane of a pair pulls its partner's
// 8 CV words with one cross-lane move each and compresses the parent.  `count` items at
// entry; ROOT on the last pair.  Every lane runs the moves (DPP needs full exec).
template <int SEG, uint32_t S>
__device__ __forceinline__ void segment_merge(uint32_t (&cv)[8], uint32_t sl, uint32_t& count) {
  if constexpr (S < (uint32_t)SEG) {
    uint32_t r[8];
#pragma unroll
    for (int w = 0; w < 8; ++w) r[w] = from_lane_above<S>(cv[w]);
    const bool left = (sl & (2u * S - 1u)) == 0u;
    if (count > 1u && left && sl / S + 1u < count) parent(cv, cv, r, count == 2u ? (uint32_t)ROOT : 0u);
    count = (count + 1u) >> 1;
    segment_merge<SEG, 2u * S>(cv, sl, count);
  }
}

// K1L: a file per SEG-lane segment (64/SEG files per wave).  Segment lane l hashes the
// CPL consecutive chunks [l*CPL, (l+1)*CPL) (CPL = the smallest power of two with
// CPL*SEG >= chunks), merges them into one subtree CV through an LDS stack column of its
// own, and the segment then merges the lanes' subtree CVs across lanes.  Aligned
// power-of-two groups make this exactly BLAKE3's left-balanced tree (level-wise
// pair-and-promote, oracle formulation 3).
//   SEG = 64: one file per wave, CPL = 1 for sampled messages (57 chunks): latency ~16 + 6
//             compression times — the smallest batches;
//   SEG = 16: four files per wave, CPL = 4: 64 + 3 block/parent compressions per lane and
//             4 cross-lane levels — ~25 % fewer wave-compressions per file, 3x the latency,
//             for mid-size batches (crossovers in profiles/r01_k1l_seg_sweep.log).
constexpr int CP_DEPTH = 3;  // CPL <= 8 -> at most 3 pending subtrees per lane

template <int SEG>
__device__ __forceinline__ void chunkpar_wave(const uint8_t* __restrict__ arena,
                                              const uint64_t* __restrict__ offs, uint64_t stride,
                                              const uint32_t* __restrict__ lens, uint32_t fixed_len,
                                              const uint64_t* __restrict__ sizes, uint64_t n,
                                              const uint32_t* __restrict__ order,
                                              uint64_t* __restrict__ keys) {
  __shared__ uint32_t stk[CP_DEPTH][8][64];  // word-major per-lane columns: conflict-free
  const uint32_t lane = threadIdx.x;
  const uint32_t sl = lane % SEG;
  const uint64_t slot = (uint64_t)blockIdx.x * (64 / SEG) + lane / SEG;
  const uint64_t f = slot < n ? (order ? (uint64_t)order[slot] : slot) : n;
  uint32_t clen = 0, nchunks = 0;
  uint64_t size = 0;
  const uint4* q = nullptr;
  if (f < n) {
    q = reinterpret_cast<const uint4*>(arena + (offs ? offs[f] : f * stride));
    clen = offs ? lens[f] : fixed_len;
    size = sizes[f];
    nchunks = (clen + 8u + 1023u) >> 10;
  }
  const bool ok = nchunks != 0 && nchunks <= CP_MAX_CHUNKS;  // caller contract: <= 104 chunks
  uint32_t cpl = 1;
  while (cpl * SEG < nchunks) cpl <<= 1;
  const bool whole = nchunks <= cpl;  // the file fits in segment lane 0: it holds the root
  const uint32_t c0 = ok ? sl * cpl : 0u;
  const uint32_t c1 = ok ? min(nchunks, c0 + cpl) : 0u;
  uint32_t cv[8] = {0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u};
  uint32_t sp = 0;
  for (uint32_t c = c0; c < c1; ++c) {
    cas_chunk_cv(q, clen, size, c, cv);  // ROOT already set for a one-chunk message
    uint32_t total = c - c0 + 1u;
    while ((total & 1u) == 0u) {
      uint32_t l[8];
      --sp;
#pragma unroll
      for (int w = 0; w < 8; ++w) l[w] = stk[sp][w][lane];
      parent(cv, l, cv, (whole && c + 1u == nchunks && sp == 0u) ? (uint32_t)ROOT : 0u);
      total >>= 1;
    }
#pragma unroll
    for (int w = 0; w < 8; ++w) stk[sp][w][lane] = cv[w];
    ++sp;
  }
  // a partial (last) group: merge its pending subtrees right to left
  if (sp > 0u) {
    --sp;
#pragma unroll
    for (int w = 0; w < 8; ++w) cv[w] = stk[sp][w][lane];
    while (sp > 0u) {
      uint32_t l[8];
      --sp;
#pragma unroll
      for (int w = 0; w < 8; ++w) l[w] = stk[sp][w][lane];
      parent(cv, l, cv, (whole && sp == 0u) ? (uint32_t)ROOT : 0u);
    }
  }
  uint32_t count = whole ? 1u : (nchunks + cpl - 1u) / cpl;  // lane subtrees of this file
  segment_merge<SEG, 1u>(cv, sl, count);
  if (f < n && sl == 0u) keys[f] = ok ? key_of(cv) : 0ull;
}

// offs == nullptr: content i at arena + i*stride with length fixed_len (the sampled
// layout); else arena + offs[i], lens[i] bytes.  One 64-lane workgroup = 64/SEG files,
// visited in `order` (nullptr = identity): ragged files sorted by chunk count so the 4
// files of a 16-lane-segment wave share one chunks-per-lane class.
template <int SEG>
__global__ void __launch_bounds__(64)
sd_cas_chunkpar_kernel(const uint8_t* __restrict__ arena, const uint64_t* __restrict__ offs,
                       uint64_t stride, const uint32_t* __restrict__ lens, uint32_t fixed_len,
                       const uint64_t* __restrict__ sizes, uint64_t n,
                       const uint32_t* __restrict__ order, uint64_t* __restrict__ keys) {
  chunkpar_wave<SEG>(arena, offs, stride, lens, fixed_len, sizes, n, order, keys);
}

// K2: whole-file path, content length <= MAX_PACKED_CONTENT_LEN, files visited in `order`.
extern "C" __global__ void __launch_bounds__(PACKED_BLOCK)
sd_cas_packed_kernel(const uint8_t* __restrict__ arena, const uint64_t* __restrict__ offs,
                     const uint32_t* __restrict__ lens, const uint64_t* __restrict__ sizes,
                     const uint32_t* __restrict__ order, uint64_t n,
                     uint64_t* __restrict__ keys) {
  __shared__ uint32_t stack_lds[PACKED_LDS_DEPTH][8][PACKED_BLOCK];
  const uint64_t t = (uint64_t)blockIdx.x * PACKED_BLOCK + threadIdx.x;
  if (t >= n) return;
  const uint32_t f = order ? order[t] : (uint32_t)t;
  const uint4* q = reinterpret_cast<const uint4*>(arena + offs[f]);
  PackedStack stk{stack_lds, threadIdx.x};
  keys[f] = cas_lane_packed(q, lens[f], sizes[f], stk);
}

}  // namespace sdcas

// ---- host launchers ----------------------------------------------------------------
namespace sdcas {

// Sort key for the K2 visiting order: (window of LEN_WINDOW consecutive files, descending
// block count).  Inside a window the lanes of a wave get (nearly) equal trip counts; the
// window keeps a wave's 64 lanes inside ~LEN_WINDOW files of the arena instead of spread
// over all of it (a global length sort scattered every wave over the whole arena and
// thrashed address translation: 4x slower on 1M files / 51 GB).
// Visiting order = STABLE sort on the descending exact BLAKE3 chunk count of the message
// (ceil((len + 8) / 1024)): the longest messages start first (no tail of late long waves),
// the lanes of a wave share the chunk count (so K2's full-chunk loop is wave-uniform and
// only the last chunk runs the generic per-block code) and, the sort being stable, the
// files of one bucket keep their arena order, so a wave's 64 lanes stay close in memory.
// Measured on 1M ragged files (profiles/r01_k2_order.txt): exact-length global sort 41 ms,
// per-window exact sort 31.7 ms, chunk buckets 17.4 ms.
// SD_K2_BLOCK_KEY=1 keys on the exact 64-B BLOCK count instead, so a wave's lanes would also
// share the last chunk's block count — measured 2.5x SLOWER (1M files: 41.2 vs 16.8 ms,
// profiles/r04_ab_keys.log): 1,664 block buckets of ~600 files spread each wave's 64 lanes over
// the whole 51 GB arena (the address-translation thrash of a global length sort), where ~104
// chunk buckets keep them within ~330 MB.  Off.
#ifndef SD_K2_BLOCK_KEY
#define SD_K2_BLOCK_KEY 0
#endif
// SD_K2_KEY_SHIFT = s: key on chunks >> s (buckets of 2^s chunk counts: a wave's lanes may
// differ by up to 2^s - 1 chunks, but a bucket's files lie 2^s times closer in the arena) —
// measured monotonically slower, 1M files 16.95 / 17.05 / 17.3 / 17.9 ms for s = 0..3
// (profiles/r04_ab_k2_keyshift.log): the lanes' balance matters, the arena distance does not
#ifndef SD_K2_KEY_SHIFT
#define SD_K2_KEY_SHIFT 0
#endif
constexpr uint32_t CHUNK_KEY_BITS = SD_K2_BLOCK_KEY ? 11 : 7;  // blocks <= 1,664 / chunks <= 104

extern "C" __global__ void __launch_bounds__(256)
sd_cas_length_keys(const uint32_t* __restrict__ lens, uint64_t n, uint64_t* __restrict__ out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    const uint64_t units = SD_K2_BLOCK_KEY ? ((uint64_t)lens[i] + 8u + 63u) >> 6
                                           : ((uint64_t)lens[i] + 8u + 1023u) >> (10 + SD_K2_KEY_SHIFT);
    out[i] = ((1ull << CHUNK_KEY_BITS) - 1) - units;
  }
}

int length_key_bits(uint64_t) { return (int)CHUNK_KEY_BITS; }

hipError_t hash_sampled(const uint8_t* content, uint64_t stride, const uint64_t* sizes,
                        uint64_t n, uint64_t* keys, hipStream_t s, uint32_t cus) {
  if (n == 0) return hipSuccess;
  const uint64_t blocks = (n + SAMPLED_BLOCK - 1) / SAMPLED_BLOCK;
  // One file per lane at 4 waves per SIMD: the 512-lane grid fills the chip in rounds of
  // two quanta (one workgroup per CU per round), the 256-lane grid in rounds of one.  The
  // wide grid is 1-2 % faster per file (profiles/r01_k1_block_ab.log) but an odd number of
  // quantum rounds leaves half its last round's SIMDs idle (3 quanta: 4.96 vs ~3.5 ms), so
  // it runs only when the batch spans an even number of quanta.
  const uint64_t quanta = cus ? (n + (uint64_t)cus * 256 - 1) / ((uint64_t)cus * 256) : 0;
  if (cus && (blocks < cus || (quanta & 1))) {
    const uint64_t nb = (n + SAMPLED_BLOCK_NARROW - 1) / SAMPLED_BLOCK_NARROW;
    sd_cas_sampled_kernel_256<<<(uint32_t)nb, SAMPLED_BLOCK_NARROW, 0, s>>>(content, stride, sizes,
                                                                           n, keys);
  } else {
    sd_cas_sampled_kernel<<<(uint32_t)blocks, SAMPLED_BLOCK, 0, s>>>(content, stride, sizes, n, keys);
  }
  return hipGetLastError();
}

hipError_t hash_sampled_regions(const uint8_t* content, uint64_t stride, const uint64_t* sizes,
                                uint64_t n, uint64_t* keys, uint32_t* rep, uint64_t* rkeys,
                                uint32_t* rfile, uint32_t* cursor, uint64_t cap, uint64_t* spill_keys,
                                uint32_t* spill_file, uint32_t* overflow, uint64_t* objects,
                                hipStream_t s, uint32_t cus) {
  if (n == 0) return hipSuccess;
  const RegionOut ro{rkeys, rfile, cursor, cap, spill_keys, spill_file, rep, overflow,
                     (unsigned long long*)objects};
  const uint64_t blocks = (n + SAMPLED_BLOCK - 1) / SAMPLED_BLOCK;
  const uint64_t quanta = cus ? (n + (uint64_t)cus * 256 - 1) / ((uint64_t)cus * 256) : 0;
  if (cus && (blocks < cus || (quanta & 1))) {  // the grid choice of hash_sampled
    const uint64_t nb = (n + SAMPLED_BLOCK_NARROW - 1) / SAMPLED_BLOCK_NARROW;
    sd_cas_sampled_group_kernel_256<<<(uint32_t)nb, SAMPLED_BLOCK_NARROW, 0, s>>>(content, stride,
                                                                                 sizes, n, keys, ro);
  } else {
    sd_cas_sampled_group_kernel<<<(uint32_t)blocks, SAMPLED_BLOCK, 0, s>>>(content, stride, sizes, n,
                                                                          keys, ro);
  }
  return hipGetLastError();
}

// A copy of pinned host memory into HBM by the shader instead of the SDMA engine (the
// path gather's streamed pieces: A/B SD_PATHS_PULL): each lane moves 16-B quads, a wave
// 1 KiB per load instruction over the host link, U quads per lane in flight.  Measured one
// piece at a time (tools/ubench_pull.hip, profiles/r04_ubench_pull.log): a 128 KiB piece
// 7.8 us with U = 1 (32 workgroups) vs 11.3 with U = 4 (8 workgroups: too few CUs issue);
// from 1 MiB on U = 4 wins (1 MiB 25.2 vs 29.0 us, 4 MiB 85.7 vs 102.6); SDMA 18 / 34 / 91 us.
// So pieces under SD_PULL_WIDE_BYTES take U = 1, larger ones SD_PULL_UNROLL.
#ifndef SD_PULL_UNROLL
#define SD_PULL_UNROLL 4  // 4 vs 1 for every piece: 100 sampled files 0.29 -> 0.26 ms
                          // (profiles/r04_ab_jobstep_pull.log)
#endif
#ifndef SD_PULL_WIDE_BYTES
#define SD_PULL_WIDE_BYTES (512u << 10)
#endif
template <int U>
__global__ void __launch_bounds__(256)
sd_pull_host(const uint4* __restrict__ src, uint4* __restrict__ dst, uint64_t quads) {
  const uint64_t step = (uint64_t)gridDim.x * 256;
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < quads; i += step * U) {
    uint4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (i + u * step < quads) v[u] = src[i + u * step];
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (i + u * step < quads) dst[i + u * step] = v[u];
  }
}

hipError_t pull_host(void* dst, const void* src, uint64_t bytes, hipStream_t s) {
  if (bytes == 0) return hipSuccess;
  if ((bytes & 15) || ((uintptr_t)dst & 15) || ((uintptr_t)src & 15))
    return hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, s);
  const uint64_t quads = bytes >> 4;
  const int u = bytes < SD_PULL_WIDE_BYTES ? 1 : SD_PULL_UNROLL;
  uint64_t blocks = (quads + 256 * u - 1) / (256 * u);
  if (blocks > 2048) blocks = 2048;
  if (u == 1)
    sd_pull_host<1><<<(uint32_t)blocks, 256, 0, s>>>((const uint4*)src, (uint4*)dst, quads);
  else
    sd_pull_host<SD_PULL_UNROLL><<<(uint32_t)blocks, 256, 0, s>>>((const uint4*)src, (uint4*)dst, quads);
  return hipGetLastError();
}

hipError_t hash_packed(const uint8_t* arena, const uint64_t* offs, const uint32_t* lens,
                       const uint64_t* sizes, const uint32_t* order, uint64_t n, uint64_t* keys,
                       hipStream_t s) {
  if (n == 0) return hipSuccess;
  const uint64_t blocks = (n + 255) / 256;
  sd_cas_packed_kernel<<<(uint32_t)blocks, 256, 0, s>>>(arena, offs, lens, sizes, order, n, keys);
  return hipGetLastError();
}

hipError_t hash_chunkpar(const uint8_t* arena, const uint64_t* offs, uint64_t stride,
                         const uint32_t* lens, uint32_t fixed_len, const uint64_t* sizes,
                         uint64_t n, uint64_t* keys, int seg, hipStream_t s,
                         const uint32_t* order) {
  if (n == 0) return hipSuccess;
  if (n >= (1ull << 31)) return hipErrorInvalidValue;
  if (seg == 16)
    sd_cas_chunkpar_kernel<16><<<(uint32_t)((n + 3) / 4), 64, 0, s>>>(
        arena, offs, stride, lens, fixed_len, sizes, n, order, keys);
  else
    sd_cas_chunkpar_kernel<64><<<(uint32_t)n, 64, 0, s>>>(arena, offs, stride, lens, fixed_len,
                                                         sizes, n, order, keys);
  return hipGetLastError();
}

hipError_t length_keys(const uint32_t* lens, uint64_t n, uint64_t* out, hipStream_t s) {
  if (n == 0) return hipSuccess;
  sd_cas_length_keys<<<(uint32_t)((n + 255) / 256), 256, 0, s>>>(lens, n, out);
  return hipGetLastError();
}

}  // namespace sdcas
