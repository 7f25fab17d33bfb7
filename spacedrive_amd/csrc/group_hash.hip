// group_hash.hip — Object grouping on gfx950 without a full sort (K4h + K5h).
//
// Replaces the grouping logic of core/src/object/file_identifier/mod.rs:98-350 (the
// unique_cas_ids HashSet :149-154, the `cas_id IN (...)` Object lookup :181-198 and the
// linear `find` over existing Objects :214-224) with the canonical contract of SURVEY.md
// §8c: rep(f) = min{ g : key(g) == key(f) }, objects = #distinct keys.
//
// The grouping never needs the keys in order — only equal keys side by side — so instead
// of an 8-pass LSD sort (256 B/key of HBM traffic, ~40 launches) it is:
//   K4h-a  sd_part_totals   per-block coarse-bucket histogram in LDS, added to the bucket
//                           totals (one atomic per bucket per block), and the prefill
//                           out[i] = val(i)                                  8 B read, 4 B write
//   K4h-b  sd_part_scatter  keys -> coarse-bucket-contiguous (mixed key, position),
//                           LDS-staged so stores are coalesced runs; each trip reserves its
//                           run inside its totals replica's sub-run of each bucket (one
//                           atomic per bucket, 1/16 of the blocks per cursor) 8 B read, 12 B write
//   K4h-c  sd_part_refine   one workgroup per coarse bucket splits it by the next bits
//                           (only above 1.44M keys)                     20 B read, 12 B write
//   K5h    sd_bucket_min    one workgroup per fine bucket: LDS hash table of the bucket's
//                           distinct keys with an atomic min of the value, then every
//                           position reads its slot's minimum; it stores only where it
//                           differs from the prefill (duplicates)            12 B read, <= 4 B write
// = 76 B/key (44 without the refine level) in 4-5 launches (a memset of the totals + the
// kernels; no [bucket][block] table and no scan: the order inside a bucket is arbitrary and
// the results do not depend on it).  Up to 1,441,792 keys (the bench's 1.31 M per GPU) the
// refine level is skipped: the 256 coarse buckets (~5,100 keys) go straight to 1,024-thread
// workgroups with 12,288-slot tables (sd_bucket_min_big).  The bucket is the top bits
// of a bijective mix of the key, so any set of DISTINCT keys spreads evenly (BLAKE3 keys are
// uniform anyway; test keys such as 0..n-1 are not), while duplicates — however many —
// share one table slot.  A bucket whose distinct keys overflow the LDS table (never for
// uniform keys: mean <= 1,536 distinct per bucket vs 3,584 allowed, ~5,100 vs 10,752 in the
// big tables) is redone by the same workgroup in a global-memory table.
//
// The same two kernels give the key-RANGE partition of the multi-GPU exchange (SURVEY §8e:
// dest = floor(key * G / 2^64)), with the bucket function applied to the raw key.
// Integer/byte work bound by HBM and LDS atomics; nothing here is reshaped into a GEMM.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "sd_debug.h"
#include "sd_group.h"
#include "sd_mix.h"

namespace sdcas {

// Every loop below moves ITEMS keys per thread per trip with all loads issued before the
// first use: one trip = one memory latency for PART_THREADS x ITEMS keys (a load-per-trip
// loop at 8 waves/CU was latency-bound at 0.45 TB/s).
constexpr int PART_THREADS = 512;
constexpr int ITEMS = 8;
constexpr uint32_t PART_TILE = PART_THREADS * ITEMS;  // 4096 keys per block trip
#ifndef SD_MIN_THREADS
#define SD_MIN_THREADS 512
#endif
#ifndef SD_MIN_TABLE
#define SD_MIN_TABLE 4096
#endif
constexpr int MIN_THREADS = SD_MIN_THREADS;
// keys per thread per trip of the fine-bucket tables (mean bucket <= 1,536 keys: one trip of
// 2,048) and whether their lookup reuses the insert's slots (A/B: DESIGN.md §2.2)
#ifndef SD_MIN_ITEMS
#define SD_MIN_ITEMS 4
#endif
#ifndef SD_MIN_KEEP_SLOT
#define SD_MIN_KEEP_SLOT 1
#endif
constexpr int MIN_ITEMS = SD_MIN_ITEMS;
#ifndef SD_ONE_TRIP_READ_FIRST
#define SD_ONE_TRIP_READ_FIRST 0
#endif
constexpr bool MIN_KEEP_SLOT = SD_MIN_KEEP_SLOT;
constexpr uint32_t TABLE = SD_MIN_TABLE;  // LDS slots per bucket (4,096: 48 KiB, 3 workgroups/CU)
constexpr uint32_t BIG_TABLE = 12288;     // sd_bucket_min_big: 144 KiB LDS, 1 workgroup/CU
constexpr int BIG_THREADS = 1024;
constexpr uint64_t BIG_MAX_KEYS = 256ull * 5632;  // mean coarse bucket <= 5,632 keys
constexpr uint32_t MAX_BUCKETS = 16384;   // LDS cursor table of the partition kernels (64 KiB)
constexpr uint64_t TARGET_PER_BUCKET = 1536;
constexpr uint64_t MAX_TABLE_ENTRIES = 2ull << 20;  // bucket-count atomics per partition pass
constexpr uint32_t TOTALS_REPL = 16;                  // interleaved copies of the bucket totals
// final buckets: 2^bits, bits = b1 (coarse, <= 10) + b2 (refine, <= 9); at the largest
// plan the mean bucket may grow to MAX_MEAN_PER_BUCKET distinct keys (LDS table fill 3,584)
constexpr uint32_t MAX_BITS = 19;
constexpr uint32_t MAX_B2 = 9;
#ifndef SD_COARSE10_KEYS
#define SD_COARSE10_KEYS 40000000
#endif
constexpr uint64_t COARSE10_KEYS = SD_COARSE10_KEYS;
constexpr uint64_t MAX_MEAN_PER_BUCKET = 2500;
// The fine-bucket tables (one workgroup per ~1,500 keys: 8,192 at 12.5 M keys, 65,536 at
// 100 M) add their distinct-key counts into OBJ_SHARDS counters, each on a 128-B line of its
// own (workgroup b into shard b % OBJ_SHARDS), summed into the Object count by one 64-lane
// launch after them.  Device-scope atomics on ONE counter complete one per ~12.8 ns: 8,192 of
// them took 105 us where the same workgroups' loads alone took 27 us, and 29 us with 64
// counters (tools/ubench_bucketload.hip, profiles/r03b_group_ab/).  SD_GROUP_OBJ_SHARDS=1:
// one counter (the A/B base).
#ifndef SD_GROUP_OBJ_SHARDS
#define SD_GROUP_OBJ_SHARDS 64
#endif
constexpr uint32_t OBJ_SHARDS = SD_GROUP_OBJ_SHARDS;
static_assert(OBJ_SHARDS >= 1 && OBJ_SHARDS <= 64, "sd_objects_sum is one wave");
constexpr uint32_t OBJ_STRIDE = 16;  // u64 words: one 128-B line per shard


// mode 0 (grouping): bucket = top bits of mix64(key), the stored key is mix64(key)
// mode 1 (range partition): bucket = floor(key * nb / 2^64), the stored key is the key
template <int MODE>
__device__ __forceinline__ uint64_t stored_key(uint64_t k) {
  return MODE == 0 ? mix64(k) : k;
}
__device__ __forceinline__ uint32_t bucket_of(uint64_t stored, uint32_t nb) {
  return (uint32_t)__umul64hi(stored, (uint64_t)nb);
}

// prefill (grouping only): out[i] = val(i) for every position, streamed with the key
// read, so that sd_bucket_min only stores where a key's minimum differs from the
// position's own value — a scattered 4-B store costs a 32-B HBM write (PMC:
// profiles/r01_pmc_group.json), and most positions are their key's first occurrence.
//
// Bucket totals: each block counts its slice in LDS and adds its counts to totals[nb]
// (one global atomic per non-empty bucket per block).  The scatter then reserves each
// trip's run inside a bucket with one atomic per bucket (order inside a bucket is
// arbitrary — the grouping never depends on it), so no [bucket][block] table and no scan
// pass are needed (measured: the scan was 3 launches / ~15 us per grouping call).  Block
// 0 also zeroes the scatter's reservation cursors and the Object counter (both are used
// only by later kernels of the chain).
// totals are kept in `repl` interleaved copies (block b adds into copy b % repl): a single
// copy took 1,024 same-address atomics per bucket at 12.5M keys (+8 us, measured); the
// scatter sums the copies.  The scatter's block b covers the same slice as the totals'
// block b, so bucket c's run is split into repl sub-runs, sub-run r sized by copy r, and
// block b reserves inside sub-run b % repl with its own cursor fill[b % repl][c]: 1/repl
// of the blocks contend on each cursor (all of them did: every block's reservation waited
// behind ~nblk same-address returning atomics).
template <int MODE, bool HAS_VALS>
__device__ void part_totals_body(const uint64_t* __restrict__ keys, uint64_t n, uint32_t nb,
                                 uint64_t per_block, uint32_t* __restrict__ totals, uint32_t repl,
                                 uint32_t* __restrict__ fill, unsigned long long* __restrict__ objects,
                                 uint32_t nobj, const uint32_t* __restrict__ vals,
                                 uint32_t* __restrict__ prefill) {
  extern __shared__ uint32_t cnt[];
  for (uint32_t b = threadIdx.x; b < nb; b += PART_THREADS) cnt[b] = 0;
  if (blockIdx.x == 0) {
    for (uint32_t b = threadIdx.x; b < repl * nb; b += PART_THREADS) fill[b] = 0;
    if (objects && threadIdx.x < nobj) objects[threadIdx.x * OBJ_STRIDE] = 0;  // the shards
  }
  __syncthreads();
  const uint64_t lo = (uint64_t)blockIdx.x * per_block;
  const uint64_t hi = lo + per_block < n ? lo + per_block : n;
  // the next trip's keys are loaded before this trip's counting atomics
  uint64_t kn[ITEMS];
  // every lane loads and stores (rows past the slice use its last row: the prefill then
  // rewrites that row's own value) — loads and stores under a branch leave the compiler
  // unable to count what is in flight, and it waits for all of it (the prefetch included)
  auto load = [&](uint64_t base) {
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) {
      const uint64_t i = base + (uint64_t)j * PART_THREADS + threadIdx.x;
      kn[j] = keys[i < hi ? i : hi - 1];
    }
  };
  if (lo < hi) load(lo);
  for (uint64_t base = lo; base < hi; base += PART_TILE) {
    uint64_t k[ITEMS];
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) k[j] = kn[j];
    load(base + PART_TILE < hi ? base + PART_TILE : hi);  // (past the end: one line, row hi - 1)
    if (MODE == 0) {  // the grouping always prefills; HAS_VALS picks the value source
#pragma unroll
      for (int j = 0; j < ITEMS; ++j) {
        const uint64_t i = base + (uint64_t)j * PART_THREADS + threadIdx.x;
        const uint64_t c = i < hi ? i : hi - 1;
        prefill[c] = HAS_VALS ? vals[c] : (uint32_t)c;
      }
    }
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) {
      const uint64_t i = base + (uint64_t)j * PART_THREADS + threadIdx.x;
      if (i < hi) atomicAdd(&cnt[bucket_of(stored_key<MODE>(k[j]), nb)], 1u);
    }
  }
  __syncthreads();
#if SD_DBG
  {  // conservation: the block's bucket counts add up to its slice
    __shared__ unsigned int dbg_sum;
    if (threadIdx.x == 0) dbg_sum = 0;
    __syncthreads();
    unsigned int part = 0;
    for (uint32_t b = threadIdx.x; b < nb; b += PART_THREADS) part += cnt[b];
    atomicAdd(&dbg_sum, part);
    __syncthreads();
    const uint64_t want = hi > lo ? hi - lo : 0;
    SD_DBG_CHECK(threadIdx.x != 0 || dbg_sum == want, "part_totals block %u counted %u of %llu keys",
                 blockIdx.x, dbg_sum, (unsigned long long)want);
  }
#endif
  uint32_t* mine = totals + (uint64_t)(blockIdx.x % repl) * nb;
  for (uint32_t b = threadIdx.x; b < nb; b += PART_THREADS)
    if (cnt[b]) atomicAdd(&mine[b], cnt[b]);
}

// Exclusive scan of cnt[0..nb) into out (both LDS) by the whole PART_THREADS block.
__device__ void lds_exclusive_scan(const uint32_t* cnt, uint32_t* out, uint32_t nb) {
  __shared__ uint32_t wsum[PART_THREADS / 64];
  const uint32_t t = threadIdx.x, lane = t & 63u, w = t >> 6;
  const uint32_t per = (nb + PART_THREADS - 1) / PART_THREADS;
  const uint32_t lo = t * per < nb ? t * per : nb, hi = lo + per < nb ? lo + per : nb;
  uint32_t sum = 0;
  for (uint32_t i = lo; i < hi; ++i) sum += cnt[i];
  uint32_t inc = sum;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(inc, o, 64);
    if (lane >= (uint32_t)o) inc += y;
  }
  if (lane == 63) wsum[w] = inc;
  __syncthreads();
  uint32_t run = inc - sum;
  for (uint32_t i = 0; i < w; ++i) run += wsum[i];
  for (uint32_t i = lo; i < hi; ++i) { out[i] = run; run += cnt[i]; }
  __syncthreads();
}

// LDS-staged scatter of one trip (<= PART_TILE keys at trip indices [0, trip_n)): the
// keys are first counting-sorted by bucket in LDS, then written so that consecutive
// lanes store consecutive slots of one bucket's run — coalesced, instead of 64 buckets
// (= 64 cache lines) per store instruction.  RESERVE: the trip's run in bucket b starts at
// bstart[b] + atomicAdd(&fill[b], count) (the coarse level: many blocks share a bucket);
// otherwise gcur[b] is this workgroup's running cursor (the refine level: one workgroup
// owns the segment).  tcnt must be zero on entry and is left zero.
constexpr uint32_t STAGED_MAX_NB = 1024;
// `prefetch` issues the next trip's loads: after this trip's reservation atomics (whose
// results are consumed after it, so the compiler's in-order wait for them does not also wait
// out the prefetch) and before its LDS scan, staging and stores.
template <bool RESERVE, bool STORE_ALL, typename BucketFn, typename Prefetch>
__device__ __forceinline__ void staged_trip(const uint64_t (&k)[ITEMS], const uint32_t (&pos)[ITEMS],
                                            uint32_t trip_n, uint32_t nb, BucketFn bfn,
                                            uint32_t* gcur, uint32_t* tcnt, uint32_t* tstart,
                                            uint64_t* skey, uint32_t* spos,
                                            const uint32_t* bstart, uint32_t* __restrict__ fill,
                                            uint64_t* __restrict__ out_keys,
                                            uint32_t* __restrict__ out_pos, Prefetch prefetch) {
  uint32_t bk[ITEMS], r[ITEMS];
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) {
    const uint32_t t = (uint32_t)j * PART_THREADS + threadIdx.x;
    bk[j] = t < trip_n ? bfn(k[j]) : 0u;
    r[j] = t < trip_n ? atomicAdd(&tcnt[bk[j]], 1u) : 0u;
  }
  __syncthreads();
  constexpr int RPT = (STAGED_MAX_NB + PART_THREADS - 1) / PART_THREADS;
  uint32_t resv[RPT];
  if (RESERVE) {
#pragma unroll
    for (int q = 0; q < RPT; ++q) {
      const uint32_t b = threadIdx.x + (uint32_t)q * PART_THREADS;
      resv[q] = b < nb && tcnt[b] ? atomicAdd(&fill[b], tcnt[b]) : 0u;
    }
  }
  prefetch();
  if (RESERVE) {
#pragma unroll
    for (int q = 0; q < RPT; ++q) {
      const uint32_t b = threadIdx.x + (uint32_t)q * PART_THREADS;
      if (b < nb && tcnt[b]) gcur[b] = bstart[b] + resv[q];
    }
  }
  lds_exclusive_scan(tcnt, tstart, nb);  // (its barriers also publish gcur)
  // conservation: the trip's per-bucket counts add up to the trip
  SD_DBG_CHECK(threadIdx.x != 0 || tstart[nb - 1] + tcnt[nb - 1] == trip_n,
               "staged trip (block %u) counted %u of %u keys", blockIdx.x,
               tstart[nb - 1] + tcnt[nb - 1], trip_n);
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) {
    const uint32_t t = (uint32_t)j * PART_THREADS + threadIdx.x;
    if (t < trip_n) {
      const uint32_t slot = tstart[bk[j]] + r[j];
      skey[slot] = k[j];
      spos[slot] = pos[j];
    }
  }
  __syncthreads();
  // STORE_ALL: every lane stores, one past the trip rewriting the trip's last row (same slot,
  // same data), so the compiler can count the stores and keeps the next trip's loads in
  // flight past them.  It pays in the 2^10-bucket coarse scatter (100 M keys: 756 -> 557 us)
  // and costs in the 2^8-bucket one (12.5 M: 62 -> 75 us); the refine is the same either way
  // (profiles/r03b_group_ab/README.md abg17-21)
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) {
    const uint32_t t0 = (uint32_t)j * PART_THREADS + threadIdx.x;
    if (STORE_ALL || t0 < trip_n) {
      const uint32_t t = t0 < trip_n ? t0 : trip_n - 1;
      const uint64_t kk = skey[t];
      const uint32_t b = bfn(kk);
      const uint32_t dest = gcur[b] + (t - tstart[b]);
      out_keys[dest] = kk;
      out_pos[dest] = spos[t];
    }
  }
  __syncthreads();
  for (uint32_t b = threadIdx.x; b < nb; b += PART_THREADS) {
    if (!RESERVE) gcur[b] += tcnt[b];
    tcnt[b] = 0;
  }
  __syncthreads();
}

// dynamic LDS of the scatter kernels: staged = bstart | tcnt | gcur | tstart | rbase | pad |
// skey | spos; above STAGED_MAX_NB buckets (range partitions into > 1,024 parts) bstart only
__host__ __device__ constexpr size_t scatter_lds_bytes(uint32_t nb) {
  return nb <= STAGED_MAX_NB ? (size_t)(5 * nb + 2) * 4 + (size_t)PART_TILE * 12 : (size_t)nb * 4;
}

// Bucket-contiguous scatter.  Every block derives the bucket starts from the totals (an
// LDS scan); block 0 publishes them (starts_out, the coarse level's segments) and, for the
// range partition, the part sizes (counts_out, u64).
template <int MODE, bool STORE_ALL>
__device__ void part_scatter_body(const uint64_t* __restrict__ keys, uint64_t n, uint32_t nb,
                                  uint64_t per_block, const uint32_t* __restrict__ totals,
                                  uint32_t repl, uint32_t* __restrict__ fill,
                                  uint64_t* __restrict__ out_keys,
                                  uint32_t* __restrict__ out_pos, uint32_t* __restrict__ starts_out,
                                  uint64_t* __restrict__ counts_out) {
  extern __shared__ uint32_t lds[];
  uint32_t* bstart = lds;
  uint32_t* tcnt = lds + nb;  // staged only; the scan below reads totals through tcnt
  uint32_t* rbase = lds + 4 * nb;  // staged: bucket start + this block's sub-run offset
  const bool staged = nb <= STAGED_MAX_NB;
  const uint32_t mine = blockIdx.x % repl;
  const uint64_t lo = (uint64_t)blockIdx.x * per_block;
  const uint64_t hi = lo + per_block < n ? lo + per_block : n;
  // the first trip's keys are loaded before the totals, so both latencies overlap
  uint64_t k[ITEMS];
  uint32_t q[ITEMS];
  // raw keys, every lane loading (rows past the slice re-read its last row; staged_trip
  // ignores them): a load under a branch, or the mix applied where it is loaded, made the
  // compiler wait for each load in turn — the next trip's loads did not overlap this one
  auto load_trip = [&](uint64_t base) {
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) {
      const uint64_t i = base + (uint64_t)j * PART_THREADS + threadIdx.x;
      k[j] = keys[i < hi ? i : hi - 1];
      q[j] = (uint32_t)i;
    }
  };
  if (staged) load_trip(lo);
  // the replicas' counts of a bucket: all TOTALS_REPL loads issued before any is summed (a
  // loop over the runtime `repl` waited out each load in turn: the prologue took 8.4 us of a
  // block's ~33, profiles/r03b_group_ab/ts_scatter.log)
  for (uint32_t b = threadIdx.x; b < nb; b += PART_THREADS) {
    uint32_t t[TOTALS_REPL];
#pragma unroll
    for (uint32_t r = 0; r < TOTALS_REPL; ++r) t[r] = r < repl ? totals[(uint64_t)r * nb + b] : 0u;
    uint32_t x = 0, pre = 0;
#pragma unroll
    for (uint32_t r = 0; r < TOTALS_REPL; ++r) {
      pre += r < mine ? t[r] : 0u;
      x += t[r];
    }
    if (staged) { tcnt[b] = x; rbase[b] = pre; }
    if (blockIdx.x == 0 && counts_out) counts_out[b] = x;
  }
  __syncthreads();
  if (staged) {
    lds_exclusive_scan(tcnt, bstart, nb);
    for (uint32_t b = threadIdx.x; b < nb; b += PART_THREADS) rbase[b] += bstart[b];
  } else if (threadIdx.x == 0) {  // > 1,024 parts (range mode only, repl = 1): sequential, rare
    uint32_t run = 0;
    for (uint32_t b = 0; b < nb; ++b) { bstart[b] = run; run += totals[b]; }
  }
  __syncthreads();
  if (blockIdx.x == 0 && starts_out)
    for (uint32_t b = threadIdx.x; b < nb; b += PART_THREADS) starts_out[b] = bstart[b];
  if (staged) {
    uint32_t* gcur = lds + 2 * nb;  // tcnt (lds + nb) is zeroed below for the trips
    uint32_t* tstart = lds + 3 * nb;
    uint64_t* skey = reinterpret_cast<uint64_t*>(lds + 5 * nb + 2);  // 20nb + 8 B: 8-B aligned
    uint32_t* spos = reinterpret_cast<uint32_t*>(skey + PART_TILE);
    uint32_t* myfill = fill + (uint64_t)mine * nb;
    for (uint32_t b = threadIdx.x; b < nb; b += PART_THREADS) tcnt[b] = 0;
    __syncthreads();
    auto bfn = [nb](uint64_t x) { return bucket_of(x, nb); };
    for (uint64_t base = lo; base < hi; base += PART_TILE) {
      uint64_t kc[ITEMS];
      uint32_t qc[ITEMS];
#pragma unroll
      for (int j = 0; j < ITEMS; ++j) { kc[j] = stored_key<MODE>(k[j]); qc[j] = q[j]; }
      const uint64_t left = hi - base;
      const uint64_t nbase = base + PART_TILE < hi ? base + PART_TILE : hi;  // (past the end: one line)
      staged_trip<true, STORE_ALL>(kc, qc, left < PART_TILE ? (uint32_t)left : PART_TILE, nb, bfn, gcur, tcnt,
                        tstart, skey, spos, rbase, myfill, out_keys, out_pos,
                        [&]() { load_trip(nbase); });  // in flight during this trip
    }
    return;
  }
  for (uint64_t base = lo; base < hi; base += PART_TILE) {
    uint64_t k[ITEMS];
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) {
      const uint64_t i = base + (uint64_t)j * PART_THREADS + threadIdx.x;
      k[j] = i < hi ? stored_key<MODE>(keys[i]) : 0;
    }
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) {
      const uint64_t i = base + (uint64_t)j * PART_THREADS + threadIdx.x;
      if (i < hi) {
        const uint32_t b = bucket_of(k[j], nb);
        const uint32_t d = bstart[b] + atomicAdd(&fill[b], 1u);
        out_keys[d] = k[j];
        out_pos[d] = (uint32_t)i;
      }
    }
  }
}

extern "C" __global__ void __launch_bounds__(PART_THREADS)
sd_part_totals_mix(const uint64_t* __restrict__ keys, uint64_t n, uint32_t nb, uint64_t per_block,
                   uint32_t* __restrict__ totals, uint32_t repl, uint32_t* __restrict__ fill,
                   unsigned long long* __restrict__ objects, uint32_t nobj,
                   const uint32_t* __restrict__ vals, uint32_t* __restrict__ prefill) {
  part_totals_body<0, false>(keys, n, nb, per_block, totals, repl, fill, objects, nobj, vals, prefill);
}
extern "C" __global__ void __launch_bounds__(PART_THREADS)
sd_part_totals_mix_vals(const uint64_t* __restrict__ keys, uint64_t n, uint32_t nb, uint64_t per_block,
                        uint32_t* __restrict__ totals, uint32_t repl, uint32_t* __restrict__ fill,
                        unsigned long long* __restrict__ objects, uint32_t nobj,
                        const uint32_t* __restrict__ vals, uint32_t* __restrict__ prefill) {
  part_totals_body<0, true>(keys, n, nb, per_block, totals, repl, fill, objects, nobj, vals, prefill);
}
extern "C" __global__ void __launch_bounds__(PART_THREADS)
sd_part_totals_range(const uint64_t* __restrict__ keys, uint64_t n, uint32_t nb, uint64_t per_block,
                     uint32_t* __restrict__ totals, uint32_t repl, uint32_t* __restrict__ fill) {
  part_totals_body<1, false>(keys, n, nb, per_block, totals, repl, fill, nullptr, 0, nullptr, nullptr);
}
extern "C" __global__ void __launch_bounds__(PART_THREADS)
sd_part_scatter_mix(const uint64_t* __restrict__ keys, uint64_t n, uint32_t nb, uint64_t per_block,
                    const uint32_t* __restrict__ totals, uint32_t repl, uint32_t* __restrict__ fill,
                    uint64_t* __restrict__ out_keys, uint32_t* __restrict__ out_pos,
                    uint32_t* __restrict__ starts_out) {
  part_scatter_body<0, false>(keys, n, nb, per_block, totals, repl, fill, out_keys, out_pos, starts_out,
                              nullptr);
}
// the same for 2^10 coarse buckets (above COARSE10_KEYS): every lane stores (STORE_ALL)
extern "C" __global__ void __launch_bounds__(PART_THREADS)
sd_part_scatter_mix_wide(const uint64_t* __restrict__ keys, uint64_t n, uint32_t nb, uint64_t per_block,
                         const uint32_t* __restrict__ totals, uint32_t repl, uint32_t* __restrict__ fill,
                         uint64_t* __restrict__ out_keys, uint32_t* __restrict__ out_pos,
                         uint32_t* __restrict__ starts_out) {
  part_scatter_body<0, true>(keys, n, nb, per_block, totals, repl, fill, out_keys, out_pos, starts_out,
                             nullptr);
}
extern "C" __global__ void __launch_bounds__(PART_THREADS)
sd_part_scatter_range(const uint64_t* __restrict__ keys, uint64_t n, uint32_t nb, uint64_t per_block,
                      const uint32_t* __restrict__ totals, uint32_t repl, uint32_t* __restrict__ fill,
                      uint64_t* __restrict__ out_keys, uint32_t* __restrict__ out_pos,
                      uint64_t* __restrict__ counts_out) {
  part_scatter_body<1, false>(keys, n, nb, per_block, totals, repl, fill, out_keys, out_pos, nullptr,
                              counts_out);
}

// Second partition level: one workgroup per coarse bucket (top b1 bits of the stored key)
// splits it by the next b2 bits, in place order -> out (bucket-contiguous within the
// segment, runs of ~PART_TILE / 2^b2 keys per trip: coalesced).  starts[c * 2^b2 + j] =
// first position of fine bucket (c, j).  A single-level partition with 2^(b1+b2) buckets
// writes runs of ~1-3 keys per bucket per block, which costs 5-10x in scattered stores
// (tools/ubench_scatter.hip); two coalesced levels move more bytes in less time.
constexpr uint32_t MAX_FINE = 1u << MAX_B2;
// refine_body: coarse bucket c's rows in_keys/in_pos[is, ie) -> out rows from os on (bucket-
// contiguous by the next b2 bits); with a spill list (the region chain: rows past the region's
// capacity), its rows of bucket c follow them (filtered, stored one by one: only inputs where
// one key repeats thousands of times have any).
__device__ __forceinline__ void refine_body(const uint64_t* __restrict__ in_keys, const uint32_t* __restrict__ in_pos,
                            uint64_t is, uint64_t ie, uint64_t os, uint32_t c, uint32_t b1,
                            uint32_t b2, uint64_t* __restrict__ out_keys,
                            uint32_t* __restrict__ out_pos, uint32_t* __restrict__ starts,
                            const uint64_t* __restrict__ spill_keys = nullptr,
                            const uint32_t* __restrict__ spill_pos = nullptr, uint64_t spill_n = 0) {
  __shared__ uint32_t cnt[MAX_FINE], gcur[MAX_FINE], tcnt[MAX_FINE], tstart[MAX_FINE];
  __shared__ uint64_t skey[PART_TILE];
  __shared__ uint32_t spos[PART_TILE];
  const uint32_t nb2 = 1u << b2;
  const uint64_t s = is, e = ie;
  if (threadIdx.x < nb2) cnt[threadIdx.x] = 0;
  __syncthreads();
  // one workgroup per coarse bucket (~1 per CU): each trip's loads are issued a trip ahead,
  // so the ~12 trips of a 12.5M-key refine do not each wait out an HBM round trip
  uint64_t kn[ITEMS];
  uint32_t qn[ITEMS];
  auto load = [&](uint64_t base, bool with_pos) {  // every lane loads (clamped, as in the totals)
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) {
      const uint64_t i = base + (uint64_t)j * PART_THREADS + threadIdx.x;
      const uint64_t c = i < e ? i : e - 1;
      kn[j] = in_keys[c];
      if (with_pos) qn[j] = in_pos[c];
    }
  };
  auto fine = [b1, b2](uint64_t x) { return (uint32_t)((x << b1) >> (64 - b2)); };
  auto mine = [b1, c](uint64_t x) { return (uint32_t)(x >> (64 - b1)) == c; };
  if (s < e) load(s, false);
  for (uint64_t base = s; base < e; base += PART_TILE) {
    uint64_t k[ITEMS];
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) k[j] = kn[j];
    load(base + PART_TILE < e ? base + PART_TILE : e, false);  // (past the end: one line, row e - 1)
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) {
      const uint64_t i = base + (uint64_t)j * PART_THREADS + threadIdx.x;
      if (i < e) atomicAdd(&cnt[fine(k[j])], 1u);
    }
  }
  for (uint64_t i = threadIdx.x; i < spill_n; i += PART_THREADS) {
    const uint64_t x = spill_keys[i];
    if (mine(x)) atomicAdd(&cnt[fine(x)], 1u);
  }
  if (s < e) load(s, true);  // the scatter pass's first trip, in flight during the plan
  __syncthreads();
#if SD_DBG
  __shared__ uint32_t dbg_end[MAX_FINE];  // where each fine bucket's cursor must end
#endif
  if (threadIdx.x == 0) {
    uint32_t run = (uint32_t)os;
    for (uint32_t j = 0; j < nb2; ++j) {
      const uint32_t x = cnt[j];
      gcur[j] = run;
      starts[(uint64_t)c * nb2 + j] = run;
      run += x;
#if SD_DBG
      dbg_end[j] = run;
#endif
    }
    SD_DBG_CHECK(spill_n || run == (uint32_t)(os + (e - s)),
                 "refine bucket %u: fine counts add to %u, segment ends at %llu", c, run,
                 (unsigned long long)(os + (e - s)));
  }
  if (threadIdx.x < nb2) tcnt[threadIdx.x] = 0;
  __syncthreads();
  for (uint64_t base = s; base < e; base += PART_TILE) {
    uint64_t k[ITEMS];
    uint32_t q[ITEMS];
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) { k[j] = kn[j]; q[j] = qn[j]; }
    load(base + PART_TILE < e ? base + PART_TILE : e, true);
    const uint64_t left = e - base;
    staged_trip<false, false>(k, q, left < PART_TILE ? (uint32_t)left : PART_TILE, nb2, fine, gcur, tcnt,
                       tstart, skey, spos, nullptr, nullptr, out_keys, out_pos, []() {});
  }
  if (spill_n) {  // (uniform) after the last trip's barrier: gcur is final for the region rows
    for (uint64_t i = threadIdx.x; i < spill_n; i += PART_THREADS) {
      const uint64_t x = spill_keys[i];
      if (mine(x)) {
        const uint32_t d = atomicAdd(&gcur[fine(x)], 1u);
        out_keys[d] = x;
        out_pos[d] = spill_pos[i];
      }
    }
    __syncthreads();
  }
  // conservation: every fine bucket's cursor advanced by exactly its count (rows written ==
  // rows counted); staged_trip's last barrier published gcur
  SD_DBG_CHECK(threadIdx.x >= nb2 || gcur[threadIdx.x] == dbg_end[threadIdx.x],
               "refine bucket %u.%u: cursor %u, expected %u", c, threadIdx.x, gcur[threadIdx.x],
               dbg_end[threadIdx.x]);
}

extern "C" __global__ void __launch_bounds__(PART_THREADS)
sd_part_refine(const uint64_t* __restrict__ in_keys, const uint32_t* __restrict__ in_pos,
               const uint32_t* __restrict__ starts1, uint32_t nb1, uint64_t n, uint32_t b1,
               uint32_t b2, uint64_t* __restrict__ out_keys, uint32_t* __restrict__ out_pos,
               uint32_t* __restrict__ starts) {
  const uint32_t c = blockIdx.x;
  const uint64_t s = starts1[c];
  const uint64_t e = c + 1 < nb1 ? starts1[c + 1] : n;
  refine_body(in_keys, in_pos, s, e, s, c, b1, b2, out_keys, out_pos, starts);
}

// Home slot of a (mixed, uniform) key in a TBL-slot table — its low bits for a power of two,
// else the high half of low32 x TBL — and the linear-probing successor.
template <uint32_t TBL>
__device__ __forceinline__ uint32_t home_slot(uint64_t k) {
  if ((TBL & (TBL - 1)) == 0) return (uint32_t)k & (TBL - 1);
  return (uint32_t)(((k & 0xFFFFFFFFull) * TBL) >> 32);
}
template <uint32_t TBL>
__device__ __forceinline__ uint32_t next_slot(uint32_t s) {
  if ((TBL & (TBL - 1)) == 0) return (s + 1) & (TBL - 1);
  return s + 1 == TBL ? 0u : s + 1;
}

// Linear-probing tables: LDS (the normal case) and global memory (overflow).
// lds_claim: the slot holding k after inserting it (CAS-first: one LDS round trip per probe;
// at the tables' fill most first probes find the slot empty — reading the slot before the
// CAS was 1-2 % slower, profiles/r02_group_ab3.log), or TBL if the table has no room;
// `fresh` counts keys this thread inserted first.  The probe loop is one exec-masked region
// per round with no branch inside: the table's value (the minimum) is updated after the
// loop, once per key.  PMC (profiles/r03b_group_ab/): the earlier form, with the atomic min
// and a read-first branch inside the loop, issued ~680 scalar instructions per wave — exec
// mask bookkeeping of the nested divergent branches — against one scalar issue per cycle
// per CU, the bucket tables' binding limit (SQ_INSTS_SALU 1.6x SQ_INSTS_VALU).
// READ_FIRST (buckets of more than one trip, i.e. a key repeated thousands of times): read
// the slot and CAS only if it is empty — one hot key otherwise serialises every lane's CAS
// on one LDS address (a key making up 40 % of 1.31 M keys: 1.19 -> 0.49 ms).
template <uint32_t TBL, bool READ_FIRST = false>
__device__ __forceinline__ uint32_t lds_claim(uint64_t* tk, uint32_t slot, uint64_t k, uint64_t empty,
                                              uint32_t& fresh) {
  uint64_t cur;
  bool done;
  if (!READ_FIRST) {
    // one-trip buckets: at most TILE < TBL keys ever enter the table, so an empty slot
    // always exists and the loop needs no probe bound (which costs a branch per round)
#pragma unroll 1
    do {
      cur = atomicCAS((unsigned long long*)&tk[slot], (unsigned long long)empty, (unsigned long long)k);
      done = cur == empty || cur == k;
      slot = done ? slot : next_slot<TBL>(slot);
    } while (!done);
    fresh += cur == empty;
    return slot;
  }
  // multi-trip buckets: up to FILL keys from earlier trips plus this trip's may exceed TBL
  uint32_t probe = 0;
#pragma unroll 1
  do {
    cur = tk[slot];
    if (cur == empty) {
      cur = atomicCAS((unsigned long long*)&tk[slot], (unsigned long long)empty, (unsigned long long)k);
      fresh += cur == empty;
    }
    done = cur == empty || cur == k;
    slot = done ? slot : next_slot<TBL>(slot);
  } while (!done && ++probe < TBL);
  return done ? slot : TBL;
}

template <uint32_t TBL>
__device__ __forceinline__ uint32_t lds_find(const uint64_t* tk, uint32_t slot, uint64_t k) {
  uint32_t probe = 0;  // present by construction; bounded anyway
#pragma unroll 1
  while (tk[slot] != k && ++probe < TBL) slot = next_slot<TBL>(slot);
  return slot;
}

// global tables are read with device-scope atomic loads: other waves of this workgroup
// CAS the slots at L2, and a plain load could be served a stale line from this CU's L1
__device__ __forceinline__ uint64_t gload(const uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ void g_insert(uint64_t* tk, uint32_t* tv, uint64_t cap, uint64_t slot,
                                         uint64_t k, uint32_t v, uint64_t empty, uint32_t& fresh) {
  for (;;) {  // cap = 2 x the bucket's keys: a free slot always exists
    uint64_t cur = gload(&tk[slot]);
    if (cur == empty) {
      const uint64_t old = atomicCAS((unsigned long long*)&tk[slot], (unsigned long long)empty,
                                     (unsigned long long)k);
      if (old == empty) { ++fresh; cur = k; } else { cur = old; }
    }
    if (cur == k) {
      atomicMin(&tv[slot], v);
      return;
    }
    slot = slot + 1 == cap ? 0 : slot + 1;
  }
}

__device__ __forceinline__ uint64_t g_find(const uint64_t* tk, uint64_t cap, uint64_t slot, uint64_t k) {
  while (gload(&tk[slot]) != k) slot = slot + 1 == cap ? 0 : slot + 1;
  return slot;
}

// One workgroup per bucket of the mixed-key partition (nb = 2^bits, bits >= 1).
// out[pos] = min{ val(j) : key(j) == key(pos) }, val(j) = vals ? vals[j] : j, stored only
// where it differs from val(pos): sd_part_totals_mix prefilled out[pos] = val(pos);
// *objects += distinct keys.  gkeys/gvals: 2n-slot overflow tables (touched only on overflow).
// A bucket of <= TILE keys (all but pathological ones) is loaded once and kept in
// registers for the lookup; larger buckets stream in TILE trips.
// KEEP_SLOT: the one-trip lookup reads the slot each key landed in during the insert
// instead of probing again (round 2 measured it slower for the 4,096-slot tables: with 8
// keys per lane it cost occupancy; at 4 keys per lane it is the same or faster,
// profiles/r03b_group_ab/).
// Regions (the fused hash + group chain): counts != nullptr — bucket b's keys are rows
// [b * region_cap, b * region_cap + min(counts[b], region_cap)) and the workgroup re-zeroes
// counts[b] after reading it (the region cursors' persistent-zero invariant).  A region whose
// count passed its capacity (a key repeated thousands of times) also takes its rows from the
// spill list (spill_keys/spill_pos[0, *spill_cnt): the rows of every full region, in no
// order; entries of other regions are skipped) — the same LDS table over region rows +
// spilled rows, so a hot key costs its own rows, not a pass over the input.  spill_cnt[0]
// (rows spilled), spill_cnt[1] (full regions, counted by the partition) and spill_cnt[2]
// (full regions done) are zero on entry; the last full region's workgroup re-zeroes them.  Only when such a region's distinct keys
// overflow the LDS table too is it regrouped exactly from the whole input rescan[0, rescan_n)
// (keys of this bucket only) in a global table of 2 x count slots carved from *spill.
template <uint32_t TBL, int THREADS, int NI, bool KEEP_SLOT>
__device__ __forceinline__ void bucket_min(uint32_t bucket, uint32_t* __restrict__ rezero,
                                           uint32_t rezero_words,
                                           const uint64_t* __restrict__ pkeys,
                                           const uint32_t* __restrict__ ppos,
                                           const uint32_t* __restrict__ vals,
                                           const uint32_t* __restrict__ starts, uint32_t nb,
                                           uint32_t bits, uint64_t n, uint32_t* __restrict__ out,
                                           unsigned long long* __restrict__ objects,
                                           uint64_t* __restrict__ gkeys,
                                           uint32_t* __restrict__ gvals,
                                           uint32_t* __restrict__ counts = nullptr,
                                           uint64_t region_cap = 0,
                                           const uint64_t* __restrict__ rescan = nullptr,
                                           uint64_t rescan_n = 0,
                                           unsigned long long* __restrict__ spill = nullptr,
                                           uint32_t count_stride = 1,
                                           const uint64_t* __restrict__ spill_keys = nullptr,
                                           const uint32_t* __restrict__ spill_pos = nullptr,
                                           uint32_t* __restrict__ spill_cnt = nullptr,
                                           uint32_t fill_limit = 0) {
  constexpr uint32_t TILE = THREADS * NI;
  // above FILL distinct keys the bucket goes to global memory; fill_limit (tests only, the
  // context's SD_CAS_TEST_TABLE_FILL) lowers it so the overflow and whole-input paths run on
  // keys K1G cannot be made to produce
  const uint32_t FILL = fill_limit && fill_limit < TBL / 8 * 7 ? fill_limit : TBL / 8 * 7;
  static_assert(TILE < TBL, "one-trip buckets must leave an empty slot (lds_claim's unbounded probe)");
  __shared__ uint64_t tk[TBL];
  __shared__ uint32_t tv[TBL];
  __shared__ uint32_t distinct;
  // overflow flag of trip t lives in ovf[t & 1] and is read after trip t+1's barrier: a
  // single flag could be raised by a fast wave's trip-(t+1) insert while a slower wave was
  // still reading it for trip t+1, splitting the waves over different barriers
  __shared__ int ovf[2];
  __shared__ uint32_t region_n, sp_n;
  __shared__ unsigned long long spill_off;
  const uint32_t b = bucket;
  // the chain's bucket totals were last read by the scatter: zero them for the next call
  // (the persistent buffer's invariant, see hash_group_min)
  if (bucket == 0)
    for (uint32_t i = threadIdx.x; i < rezero_words; i += THREADS) rezero[i] = 0;
  // rows [s, e_rows) are the bucket's own; [e_rows, e) index the spill list (regions only)
  uint64_t s, e, e_rows;
  if (counts) {
    if (threadIdx.x == 0) {
      region_n = counts[b * count_stride];
      counts[b * count_stride] = 0;
      uint32_t c = 0;
      if (spill_cnt && region_n > region_cap) {
        // only full regions read the spill count; the partition counted them (spill_cnt[1]),
        // so the last of them re-zeroes the three counters — regions that fit pay nothing
        c = __hip_atomic_load(spill_cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const uint32_t full = __hip_atomic_load(spill_cnt + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __threadfence();  // the reads land before this workgroup counts itself done
        if (atomicAdd(spill_cnt + 2, 1u) == full - 1) {
          spill_cnt[0] = 0;
          spill_cnt[1] = 0;
          spill_cnt[2] = 0;
        }
      }
      sp_n = c;
    }
    __syncthreads();
    s = (uint64_t)b * region_cap;
    e = e_rows = s + (region_n < region_cap ? region_n : region_cap);
    if (rescan && region_n > region_cap) {
      if (spill_keys) e += sp_n;  // region rows + the spilled rows of this region
      else e = e_rows = s;        // (uniform) no spill list: straight to the whole-input regroup
    }
  } else {
    s = starts[b];
    e = e_rows = b + 1 < nb ? starts[b + 1] : n;
  }
  // every stored key of this bucket has top bits == b, so a key from bucket b^1 is never
  // stored; the table is initialised while the bucket bounds are in flight
  const uint64_t empty = (uint64_t)(b ^ 1u) << (64 - bits);
  // row i of the bucket: its own rows, then the spill entries (other regions' read as empty)
  const bool spilled = e != e_rows;  // (uniform)
  auto load = [&](uint64_t i, uint64_t& kk, uint32_t& pp) {
    if (!spilled) {  // every bucket but a full region's: a predicated load
      kk = i < e ? pkeys[i] : empty;
      pp = i < e ? ppos[i] : 0u;
    } else if (i < e_rows) {
      kk = pkeys[i];
      pp = ppos[i];
    } else if (i < e) {
      kk = spill_keys[i - e_rows];
      pp = spill_pos[i - e_rows];
      if ((uint32_t)(kk >> (64 - bits)) != b) { kk = empty; pp = 0u; }
    } else {
      kk = empty;
      pp = 0u;
    }
  };
  for (uint32_t i = threadIdx.x; i < TBL; i += THREADS) { tk[i] = empty; tv[i] = 0xFFFFFFFFu; }
  if (threadIdx.x == 0) { distinct = 0; ovf[0] = 0; ovf[1] = 0; }
  // a region past its capacity: exact from its rows + spill in LDS, else from the whole input
  const bool full = counts && rescan && region_n > region_cap;
  const bool whole = full && !spill_keys;
  if (s == e && !whole) return;  // uniform for the whole workgroup
#if SD_DBG
  __shared__ unsigned int dbg_seen;  // keys inserted: must be the bucket's e - s
  if (threadIdx.x == 0) dbg_seen = 0;
#endif
  uint64_t k[NI];
  uint32_t p[NI], v[NI], sl[NI];
  uint32_t trip = 0;
  for (uint64_t base = s; base < e; base += TILE, ++trip) {
#pragma unroll
    for (int j = 0; j < NI; ++j) load(base + (uint64_t)j * THREADS + threadIdx.x, k[j], p[j]);
#pragma unroll
    for (int j = 0; j < NI; ++j) v[j] = (vals && k[j] != empty) ? vals[p[j]] : p[j];
    __syncthreads();  // table initialised (first trip) / the previous trip's flag visible
    if (ovf[(trip + 1) & 1]) break;  // raised by trip - 1 (ovf[1] = 0 on the first trip)
    uint32_t fresh = 0;
    bool ok = true;
    // -> each key's slot (kept for the one-trip lookup), then its minimum
    if (e - s <= TILE) {
#pragma unroll
      for (int j = 0; j < NI; ++j)
        if (k[j] != empty)
          sl[j] = lds_claim<TBL, SD_ONE_TRIP_READ_FIRST>(tk, home_slot<TBL>(k[j]), k[j], empty, fresh);
#pragma unroll
      for (int j = 0; j < NI; ++j) {
        if (k[j] != empty && sl[j] < TBL) atomicMin(&tv[sl[j]], v[j]);
        ok &= k[j] == empty || sl[j] < TBL;
      }
    } else {
#pragma unroll
      for (int j = 0; j < NI; ++j)
        if (k[j] != empty) sl[j] = lds_claim<TBL, true>(tk, home_slot<TBL>(k[j]), k[j], empty, fresh);
#pragma unroll
      for (int j = 0; j < NI; ++j) {
        if (k[j] != empty && sl[j] < TBL && tv[sl[j]] > v[j]) atomicMin(&tv[sl[j]], v[j]);
        ok &= k[j] == empty || sl[j] < TBL;
      }
    }
    // the wave's fresh keys summed by ballots (fresh <= NI <= 15 per lane), one returning LDS
    // atomic per wave instead of one per lane on one address: the insert phase halved (fine
    // tables 3.9 -> 1.8 us, big 6.6 -> 3.4 us per workgroup); sd_bucket_min at 12.5 M keys
    // 106.6 -> 87.8 us once its Object count is sharded (before that the one device counter
    // bound the kernel either way, profiles/r03b_group_ab/README.md abg16)
    static_assert(NI <= 15, "fresh fits 4 bits");
    const uint32_t wfresh = __popcll(__ballot(fresh & 1u)) + 2u * __popcll(__ballot(fresh & 2u)) +
                            4u * __popcll(__ballot(fresh & 4u)) + 8u * __popcll(__ballot(fresh & 8u));
    if ((threadIdx.x & 63u) == 0 && wfresh && atomicAdd(&distinct, wfresh) + wfresh > FILL)
      ovf[trip & 1] = 1;
    if (!ok) ovf[trip & 1] = 1;
#if SD_DBG
    unsigned int seen = 0;
#pragma unroll
    for (int j = 0; j < NI; ++j) seen += k[j] != empty;
    if (seen) atomicAdd(&dbg_seen, seen);
#endif
  }
  __syncthreads();
  const bool overflow = whole || (ovf[0] | ovf[1]);
  SD_DBG_CHECK(threadIdx.x != 0 || overflow || spilled ||
                   (dbg_seen == e - s && distinct <= e - s),
               "bucket %u: inserted %u of %llu keys, %u distinct", b, dbg_seen,
               (unsigned long long)(e - s), distinct);
  if (!overflow) {
    if (e - s <= TILE) {  // the one trip's keys and their slots are still in registers
#pragma unroll
      for (int j = 0; j < NI; ++j)
        if (k[j] != empty) {
          const uint32_t mv =
              tv[KEEP_SLOT ? sl[j] : lds_find<TBL>(tk, home_slot<TBL>(k[j]), k[j])];
          if (mv != v[j]) out[p[j]] = mv;  // out[] was prefilled with the own value
        }
    } else {
      for (uint64_t base = s; base < e; base += TILE) {
#pragma unroll
        for (int j = 0; j < NI; ++j) load(base + (uint64_t)j * THREADS + threadIdx.x, k[j], p[j]);
#pragma unroll
        for (int j = 0; j < NI; ++j)
          if (k[j] != empty) {
            const uint32_t mv = tv[lds_find<TBL>(tk, home_slot<TBL>(k[j]), k[j])];
            if (mv != (vals ? vals[p[j]] : p[j])) out[p[j]] = mv;
          }
      }
    }
    if (threadIdx.x == 0) atomicAdd(objects, (unsigned long long)distinct);
    return;
  }
  // Overflow: redo the bucket in its own 2m-slot global table (load <= 1/2); a region past
  // its capacity (its rows + spill may exceed the region's own 2 x cap slots) from the whole
  // input, in 2 x count slots carved from *spill
  const bool wh = whole || full;
  const uint64_t m = wh ? (uint64_t)region_n : e - s, cap = 2 * m;
  if (wh && threadIdx.x == 0) spill_off = atomicAdd(spill, (unsigned long long)cap);
  __syncthreads();
  uint64_t* gk = gkeys + (wh ? (uint64_t)spill_off : 2 * s);
  uint32_t* gv = gvals + (wh ? (uint64_t)spill_off : 2 * s);
  for (uint64_t i = threadIdx.x; i < cap; i += THREADS) { gk[i] = empty; gv[i] = 0xFFFFFFFFu; }
  if (threadIdx.x == 0) distinct = 0;
  __threadfence();
  __syncthreads();
  const uint64_t lo = wh ? 0 : s, hi = wh ? rescan_n : e;
  uint32_t fresh = 0;
  for (uint64_t i = lo + threadIdx.x; i < hi; i += THREADS) {
    const uint64_t kk = wh ? mix64(rescan[i]) : pkeys[i];
    if (wh && (uint32_t)(kk >> (64 - bits)) != b) continue;
    const uint32_t pp = wh ? (uint32_t)i : ppos[i];
    g_insert(gk, gv, cap, (kk & 0xFFFFFFFFull) % cap, kk, vals ? vals[pp] : pp, empty, fresh);
  }
  if (fresh) atomicAdd(&distinct, fresh);
  __threadfence();
  __syncthreads();
  for (uint64_t i = lo + threadIdx.x; i < hi; i += THREADS) {
    const uint64_t kk = wh ? mix64(rescan[i]) : pkeys[i];
    if (wh && (uint32_t)(kk >> (64 - bits)) != b) continue;
    const uint32_t pp = wh ? (uint32_t)i : ppos[i];
    const uint64_t slot = g_find(gk, cap, (kk & 0xFFFFFFFFull) % cap, kk);
    const uint32_t mv = __hip_atomic_load(&gv[slot], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (mv != (vals ? vals[pp] : pp)) out[pp] = mv;
  }
  if (threadIdx.x == 0) atomicAdd(objects, (unsigned long long)distinct);
}


extern "C" __global__ void __launch_bounds__(MIN_THREADS)
sd_bucket_min(const uint64_t* __restrict__ pkeys, const uint32_t* __restrict__ ppos,
              const uint32_t* __restrict__ vals, const uint32_t* __restrict__ starts, uint32_t nb,
              uint32_t bits, uint64_t n, uint32_t* __restrict__ out,
              unsigned long long* __restrict__ objects, uint64_t* __restrict__ gkeys,
              uint32_t* __restrict__ gvals, uint32_t* __restrict__ rezero, uint32_t rezero_words) {
  bucket_min<TABLE, MIN_THREADS, MIN_ITEMS, MIN_KEEP_SLOT>(blockIdx.x, rezero, rezero_words, pkeys, ppos,
                                                          vals, starts, nb, bits, n, out,
                                                          objects + (blockIdx.x % OBJ_SHARDS) * OBJ_STRIDE,
                                                          gkeys, gvals);
}

// Small batches (<= BIG_MAX_KEYS): the 2^8 coarse buckets of the first partition level
// (~5,100 keys at 1.31 M) go straight to 1,024-thread workgroups with a 12,288-slot table
// (144 KiB LDS, one per CU; fill ~0.42 — 8,192 slots at fill 0.625 probed ~4 times per
// insert and ran 3 % slower, profiles/r02_group_ab2.log) — no refine level, one launch and
// 24 B/key fewer.
extern "C" __global__ void __launch_bounds__(BIG_THREADS)
sd_bucket_min_big(const uint64_t* __restrict__ pkeys, const uint32_t* __restrict__ ppos,
                  const uint32_t* __restrict__ vals, const uint32_t* __restrict__ starts,
                  uint32_t nb, uint32_t bits, uint64_t n, uint32_t* __restrict__ out,
                  unsigned long long* __restrict__ objects, uint64_t* __restrict__ gkeys,
                  uint32_t* __restrict__ gvals, uint32_t* __restrict__ rezero,
                  uint32_t rezero_words) {
  bucket_min<BIG_TABLE, BIG_THREADS, ITEMS, true>(blockIdx.x, rezero, rezero_words, pkeys, ppos, vals,
                                           starts, nb, bits, n, out, objects, gkeys, gvals);
}

// The fused chain's bucket tables: one workgroup per region (the coarse buckets K1G wrote),
// straight from the regions — no totals, scatter or refine launch.  2^9 regions: 512 lanes x 7
// keys over a 6,144-slot table (72 KiB, two workgroups per CU; a region of <= 3,584 keys, every
// batch up to BIG_MAX_KEYS, is one trip).  2^8 regions: the 1,024-lane big table.  A region
// whose cursor passed its capacity (K1G appended the rows it could not store to the set's
// spill list) takes its rows from the region and the spill list (bucket_min); only if its
// distinct keys overflow the LDS table too is it regrouped from the whole key array `keys`
// (K1G's output, unmixed) in a global table carved from the set's 2 x rows overflow slots by
// objects[1] (zeroed by K1G): the grouping is exact whatever the key distribution, with no
// host regroup.
constexpr uint32_t REG_TABLE = REGION_BITS >= 9 ? 6144 : BIG_TABLE;
constexpr int REG_THREADS = REGION_BITS >= 9 ? 512 : BIG_THREADS;
constexpr int REG_ITEMS = REGION_BITS >= 9 ? 7 : ITEMS;
extern "C" __global__ void __launch_bounds__(REG_THREADS)
sd_bucket_min_regions(const uint64_t* __restrict__ rkeys, const uint32_t* __restrict__ rfile,
                      uint32_t* __restrict__ cursor, uint64_t cap, uint32_t* __restrict__ out,
                      unsigned long long* __restrict__ objects, uint64_t* __restrict__ gkeys,
                      uint32_t* __restrict__ gvals, const uint64_t* __restrict__ keys, uint64_t n,
                      const uint64_t* __restrict__ spill_keys, const uint32_t* __restrict__ spill_file,
                      uint32_t fill_limit) {
  bucket_min<REG_TABLE, REG_THREADS, REG_ITEMS, true>(blockIdx.x, nullptr, 0, rkeys, rfile, nullptr,
                                                      nullptr, REGIONS, REGION_BITS, 0, out, objects,
                                                      gkeys, gvals, cursor, cap, keys, n, objects + 1,
                                                      1, spill_keys, spill_file,
                                                      cursor + REGION_SPILL_WORD, fill_limit);
}

// The standalone chain for small batches (<= BIG_MAX_KEYS keys, default plan): the keys
// already in HBM go through K1G's region epilogue — one pass into the fixed-capacity regions
// (mixed key, row), out[] prefilled, one LDS histogram per 4,096 keys and one reservation
// atomic per (workgroup, non-empty region) — then the region tables: two launches instead
// of totals + scatter + tables.  A region past its capacity (a key repeated thousands of
// times) keeps counting in its cursor and its extra rows go to the spill list (one
// reservation per workgroup that has any), which its table workgroup reads after the region
// rows.  cursor: REGIONS u32 CURSOR_STRIDE apart (own 128-B lines), then at REGIONS *
// CURSOR_STRIDE the spill count, the full-region count and the tables' done count; all zero
// on entry (the tables re-zero them).
#ifndef SD_REGION_CURSOR_STRIDE
#define SD_REGION_CURSOR_STRIDE 32
#endif
constexpr uint32_t CURSOR_STRIDE = SD_REGION_CURSOR_STRIDE;
constexpr int RPART_THREADS = 512;
constexpr int RPART_ITEMS = 8;
constexpr uint32_t RPART_TILE = RPART_THREADS * RPART_ITEMS;
extern "C" __global__ void __launch_bounds__(RPART_THREADS)
sd_region_partition(const uint64_t* __restrict__ keys, const uint32_t* __restrict__ vals, uint64_t n,
                    uint64_t* __restrict__ rkeys, uint32_t* __restrict__ rfile,
                    uint32_t* __restrict__ cursor, uint64_t cap, uint32_t* __restrict__ out,
                    unsigned long long* __restrict__ objects, unsigned long long* __restrict__ spill,
                    uint64_t* __restrict__ spill_keys, uint32_t* __restrict__ spill_file) {
  static_assert(RPART_THREADS == PART_THREADS, "lds_exclusive_scan runs on PART_THREADS lanes");
  __shared__ uint32_t tcnt[REGIONS], tstart[REGIONS], gbase[REGIONS], spoff[REGIONS];
  __shared__ uint32_t sp_local, sp_base;
  __shared__ uint64_t skey[RPART_TILE];
  __shared__ uint32_t sfile[RPART_TILE];
  const uint64_t b0 = (uint64_t)blockIdx.x * RPART_TILE;
  const uint32_t tile_n = n - b0 < RPART_TILE ? (uint32_t)(n - b0) : RPART_TILE;
  uint64_t k[RPART_ITEMS];
  uint32_t v[RPART_ITEMS], r[RPART_ITEMS];
  // clamped, unconditional loads (no per-lane branch around them: one wait for all)
#pragma unroll
  for (int j = 0; j < RPART_ITEMS; ++j) {
    const uint64_t i = b0 + (uint64_t)j * RPART_THREADS + threadIdx.x;
    k[j] = keys[i < n ? i : n - 1];
  }
  if (vals) {
#pragma unroll
    for (int j = 0; j < RPART_ITEMS; ++j) {
      const uint64_t i = b0 + (uint64_t)j * RPART_THREADS + threadIdx.x;
      v[j] = vals[i < n ? i : n - 1];
    }
  }
  for (uint32_t i = threadIdx.x; i < REGIONS; i += RPART_THREADS) tcnt[i] = 0;
  if (threadIdx.x == 0) sp_local = 0;
  if (blockIdx.x == 0 && threadIdx.x == 0) { *objects = 0; *spill = 0; }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < RPART_ITEMS; ++j) {
    const uint32_t t = (uint32_t)j * RPART_THREADS + threadIdx.x;
    k[j] = mix64(k[j]);
    if (t < tile_n) {
      r[j] = atomicAdd(&tcnt[(uint32_t)(k[j] >> (64 - REGION_BITS))], 1u);
      out[b0 + t] = vals ? v[j] : (uint32_t)(b0 + t);
    }
  }
  __syncthreads();
  // one reservation per non-empty region, then the tile counting-sorted by region in LDS so
  // that consecutive lanes store consecutive rows of one region's run
  // rows past a region's capacity: the tile's run of them per region (spoff) inside one
  // spill reservation per workgroup
  for (uint32_t b = threadIdx.x; b < REGIONS; b += RPART_THREADS) {
    const uint32_t h = tcnt[b];
    const uint32_t g = h ? atomicAdd(&cursor[b * CURSOR_STRIDE], h) : 0u;
    gbase[b] = g;
    const uint64_t lo = g > cap ? g : cap;
    const uint32_t sp = g + h > lo ? (uint32_t)(g + h - lo) : 0u;
    spoff[b] = sp ? atomicAdd(&sp_local, sp) : 0u;
    if (g <= cap && g + h > cap) atomicAdd(&cursor[REGIONS * CURSOR_STRIDE + 1], 1u);  // it filled
  }
  lds_exclusive_scan(tcnt, tstart, REGIONS);  // (its barriers also publish gbase, spoff)
  if (sp_local) {  // (uniform) this tile overflowed a region
    if (threadIdx.x == 0) sp_base = atomicAdd(&cursor[REGIONS * CURSOR_STRIDE], sp_local);
    __syncthreads();
  }
  // conservation: the tile's per-region counts add up to the tile
  SD_DBG_CHECK(threadIdx.x != 0 || tstart[REGIONS - 1] + tcnt[REGIONS - 1] == tile_n,
               "region partition (block %u) counted %u of %u keys", blockIdx.x,
               tstart[REGIONS - 1] + tcnt[REGIONS - 1], tile_n);
#pragma unroll
  for (int j = 0; j < RPART_ITEMS; ++j) {
    const uint32_t t = (uint32_t)j * RPART_THREADS + threadIdx.x;
    if (t < tile_n) {
      const uint32_t slot = tstart[(uint32_t)(k[j] >> (64 - REGION_BITS))] + r[j];
      skey[slot] = k[j];
      sfile[slot] = (uint32_t)(b0 + t);
    }
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < RPART_ITEMS; ++j) {
    const uint32_t t = (uint32_t)j * RPART_THREADS + threadIdx.x;
    if (t < tile_n) {
      const uint64_t kk = skey[t];
      const uint32_t b = (uint32_t)(kk >> (64 - REGION_BITS));
      const uint64_t o = (uint64_t)gbase[b] + (t - tstart[b]);
      if (o < cap) {
        rkeys[(uint64_t)b * cap + o] = kk;
        rfile[(uint64_t)b * cap + o] = sfile[t];
      } else {  // past the capacity: the spill list (the region's table reads it)
        const uint64_t d = (uint64_t)sp_base + spoff[b] + (o - (gbase[b] > cap ? gbase[b] : cap));
        spill_keys[d] = kk;
        spill_file[d] = sfile[t];
      }
    }
  }
}

extern "C" __global__ void __launch_bounds__(REG_THREADS)
sd_bucket_min_regions_keys(const uint64_t* __restrict__ rkeys, const uint32_t* __restrict__ rfile,
                           uint32_t* __restrict__ cursor, uint64_t cap,
                           const uint64_t* __restrict__ keys, const uint32_t* __restrict__ vals,
                           uint64_t n, uint32_t* __restrict__ out,
                           unsigned long long* __restrict__ objects, uint64_t* __restrict__ gkeys,
                           uint32_t* __restrict__ gvals, unsigned long long* __restrict__ spill,
                           const uint64_t* __restrict__ spill_keys,
                           const uint32_t* __restrict__ spill_file) {
  bucket_min<REG_TABLE, REG_THREADS, REG_ITEMS, true>(blockIdx.x, nullptr, 0, rkeys, rfile, vals,
                                                      nullptr, REGIONS, REGION_BITS, 0, out, objects,
                                                      gkeys, gvals, cursor, cap, keys, n, spill,
                                                      CURSOR_STRIDE, spill_keys, spill_file,
                                                      cursor + REGIONS * CURSOR_STRIDE);
}

// The region chain above 1.44 M keys (default plan): one pass of the keys into 2^b1 fixed-
// capacity coarse regions (sd_region_partition_big: 8,192 keys per 1,024-lane workgroup,
// LDS-staged), the refine over each region (its output segment starts at the sum of the
// preceding regions' counts), then the fine tables — no totals pass.  Rows past a region's
// capacity go to a spill list (one reservation per workgroup that has any) that the refine of
// their region reads after its region rows.  The cursors (CURSOR_STRIDE apart) and the spill
// count live in the persistent totals buffer, zero on entry; the tables re-zero them.
#ifndef SD_RBIG_THREADS
#define SD_RBIG_THREADS 1024
#endif
#ifndef SD_RBIG_ITEMS
#define SD_RBIG_ITEMS 8
#endif
#ifndef SD_RBIG_MAX_NB
#define SD_RBIG_MAX_NB 256
#endif
constexpr int RBIG_THREADS = SD_RBIG_THREADS;
constexpr int RBIG_ITEMS = SD_RBIG_ITEMS;
constexpr uint32_t RBIG_TILE = RBIG_THREADS * RBIG_ITEMS;
constexpr uint32_t RBIG_MAX_NB = SD_RBIG_MAX_NB;

// Exclusive scan of cnt[0..nb) into out (both LDS) by a THREADS-lane block.
template <int THREADS>
__device__ void lds_exclusive_scan_t(const uint32_t* cnt, uint32_t* out, uint32_t nb) {
  __shared__ uint32_t wsum[THREADS / 64];
  const uint32_t t = threadIdx.x, lane = t & 63u, w = t >> 6;
  const uint32_t per = (nb + THREADS - 1) / THREADS;
  const uint32_t lo = t * per < nb ? t * per : nb, hi = lo + per < nb ? lo + per : nb;
  uint32_t sum = 0;
  for (uint32_t i = lo; i < hi; ++i) sum += cnt[i];
  uint32_t inc = sum;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(inc, o, 64);
    if (lane >= (uint32_t)o) inc += y;
  }
  if (lane == 63) wsum[w] = inc;
  __syncthreads();
  uint32_t run = inc - sum;
  for (uint32_t i = 0; i < w; ++i) run += wsum[i];
  for (uint32_t i = lo; i < hi; ++i) { out[i] = run; run += cnt[i]; }
  __syncthreads();
}

extern "C" __global__ void __launch_bounds__(RBIG_THREADS)
sd_region_partition_big(const uint64_t* __restrict__ keys, const uint32_t* __restrict__ vals,
                        uint64_t n, uint32_t rbits, uint64_t* __restrict__ rkeys,
                        uint32_t* __restrict__ rfile, uint32_t* __restrict__ cursor, uint64_t cap,
                        uint32_t* __restrict__ out, unsigned long long* __restrict__ shards,
                        uint32_t nshards, uint32_t* __restrict__ spill_cnt,
                        uint64_t* __restrict__ spill_keys, uint32_t* __restrict__ spill_pos) {
  __shared__ uint32_t tcnt[RBIG_MAX_NB], tstart[RBIG_MAX_NB], gbase[RBIG_MAX_NB];
  __shared__ uint64_t skey[RBIG_TILE];
  __shared__ uint32_t sfile[RBIG_TILE];
  __shared__ uint32_t sp_n, sp_i, sp_base;
  const uint32_t nb = 1u << rbits;
  const uint64_t b0 = (uint64_t)blockIdx.x * RBIG_TILE;
  const uint32_t tile_n = n - b0 < RBIG_TILE ? (uint32_t)(n - b0) : RBIG_TILE;
  uint64_t k[RBIG_ITEMS];
  uint32_t v[RBIG_ITEMS], r[RBIG_ITEMS];
#pragma unroll
  for (int j = 0; j < RBIG_ITEMS; ++j) {
    const uint64_t i = b0 + (uint64_t)j * RBIG_THREADS + threadIdx.x;
    k[j] = keys[i < n ? i : n - 1];
  }
  if (vals) {
#pragma unroll
    for (int j = 0; j < RBIG_ITEMS; ++j) {
      const uint64_t i = b0 + (uint64_t)j * RBIG_THREADS + threadIdx.x;
      v[j] = vals[i < n ? i : n - 1];
    }
  }
  for (uint32_t i = threadIdx.x; i < nb; i += RBIG_THREADS) tcnt[i] = 0;
  if (threadIdx.x == 0) { sp_n = 0; sp_i = 0; }
  if (blockIdx.x == 0 && threadIdx.x < nshards) shards[threadIdx.x * OBJ_STRIDE] = 0;
  __syncthreads();
#pragma unroll
  for (int j = 0; j < RBIG_ITEMS; ++j) {
    const uint32_t t = (uint32_t)j * RBIG_THREADS + threadIdx.x;
    k[j] = mix64(k[j]);
    if (t < tile_n) {
      r[j] = atomicAdd(&tcnt[(uint32_t)(k[j] >> (64 - rbits))], 1u);
      out[b0 + t] = vals ? v[j] : (uint32_t)(b0 + t);
    }
  }
  __syncthreads();
  for (uint32_t b = threadIdx.x; b < nb; b += RBIG_THREADS) {
    const uint32_t h = tcnt[b];
    const uint32_t g = h ? atomicAdd(&cursor[b * CURSOR_STRIDE], h) : 0u;
    gbase[b] = g;
    if ((uint64_t)g + h > cap) atomicAdd(&sp_n, (uint32_t)((uint64_t)g + h - (g > cap ? g : cap)));
  }
  lds_exclusive_scan_t<RBIG_THREADS>(tcnt, tstart, nb);  // (its barriers publish gbase, sp_n)
  SD_DBG_CHECK(threadIdx.x != 0 || tstart[nb - 1] + tcnt[nb - 1] == tile_n,
               "region partition (block %u) counted %u of %u keys", blockIdx.x,
               tstart[nb - 1] + tcnt[nb - 1], tile_n);
  if (threadIdx.x == 0 && sp_n) sp_base = atomicAdd(spill_cnt, sp_n);
#pragma unroll
  for (int j = 0; j < RBIG_ITEMS; ++j) {
    const uint32_t t = (uint32_t)j * RBIG_THREADS + threadIdx.x;
    if (t < tile_n) {
      const uint32_t slot = tstart[(uint32_t)(k[j] >> (64 - rbits))] + r[j];
      skey[slot] = k[j];
      sfile[slot] = (uint32_t)(b0 + t);
    }
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < RBIG_ITEMS; ++j) {
    const uint32_t t = (uint32_t)j * RBIG_THREADS + threadIdx.x;
    if (t < tile_n) {
      const uint64_t kk = skey[t];
      const uint32_t b = (uint32_t)(kk >> (64 - rbits));
      const uint64_t o = (uint64_t)gbase[b] + (t - tstart[b]);
      if (o < cap) {
        rkeys[(uint64_t)b * cap + o] = kk;
        rfile[(uint64_t)b * cap + o] = sfile[t];
      } else {
        const uint32_t d = sp_base + atomicAdd(&sp_i, 1u);
        spill_keys[d] = kk;
        spill_pos[d] = sfile[t];
      }
    }
  }
}

// The refine of region c: its output segment starts at the preceding regions' counts.
extern "C" __global__ void __launch_bounds__(PART_THREADS)
sd_part_refine_regions(const uint64_t* __restrict__ rkeys, const uint32_t* __restrict__ rfile,
                       const uint32_t* __restrict__ cursor, uint64_t cap, uint32_t b1, uint32_t b2,
                       const uint32_t* __restrict__ spill_cnt,
                       const uint64_t* __restrict__ spill_keys,
                       const uint32_t* __restrict__ spill_pos, uint64_t* __restrict__ out_keys,
                       uint32_t* __restrict__ out_pos, uint32_t* __restrict__ starts) {
  __shared__ uint32_t wsum[PART_THREADS / 64];
  const uint32_t c = blockIdx.x;
  uint32_t part = 0;
  for (uint32_t b = threadIdx.x; b < c; b += PART_THREADS) part += cursor[b * CURSOR_STRIDE];
  const uint32_t cnt = cursor[c * CURSOR_STRIDE];
  const uint32_t sp = cnt > cap ? *spill_cnt : 0u;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) part += __shfl_xor(part, o, 64);
  if ((threadIdx.x & 63u) == 0) wsum[threadIdx.x >> 6] = part;
  __syncthreads();
  uint32_t os = 0;
#pragma unroll
  for (int w = 0; w < PART_THREADS / 64; ++w) os += wsum[w];
  const uint64_t is = (uint64_t)c * cap;
  refine_body(rkeys, rfile, is, is + (cnt < cap ? cnt : cap), os, c, b1, b2, out_keys, out_pos, starts,
              spill_keys, spill_pos, sp);
}

}  // namespace sdcas

// ---- host launchers ----------------------------------------------------------------
namespace sdcas {

static inline size_t al256(size_t x) { return (x + 255) / 256 * 256; }

// Fixed region capacity of the fused chain for a batch of n uniform keys: the mean coarse
// bucket + 8 standard deviations (binomial) + 64 rows (the exchange's fixed_capacity rule).
uint64_t region_capacity(uint64_t n) {
  const double mean = (double)n / REGIONS;
  const double var = mean * (1.0 - 1.0 / REGIONS);
  uint64_t sd = 1;
  while ((double)(sd * sd) < var) ++sd;
  return (uint64_t)mean + 1 + 8 * sd + 64;
}

bool region_group_supported(uint64_t n) { return n > 0 && n <= BIG_MAX_KEYS; }

// workspace: rkeys | rfile | global overflow tables (2 slots per region row) | spill list
// (keys, files: n rows at most)
size_t region_group_workspace_bytes(uint64_t n) {
  const uint64_t rows = (uint64_t)REGIONS * region_capacity(n);
  return al256(rows * 8) + al256(rows * 4) + al256(2 * rows * 8) + al256(2 * rows * 4) +
         al256(n * 8) + al256(n * 4);
}

void region_group_layout(void* ws, uint64_t n, uint64_t** rkeys, uint32_t** rfile, uint64_t** gkeys,
                         uint32_t** gvals, uint64_t** spill_keys, uint32_t** spill_file) {
  const uint64_t rows = (uint64_t)REGIONS * region_capacity(n);
  char* q = (char*)ws;
  *rkeys = (uint64_t*)q; q += al256(rows * 8);
  *rfile = (uint32_t*)q; q += al256(rows * 4);
  *gkeys = (uint64_t*)q; q += al256(2 * rows * 8);
  *gvals = (uint32_t*)q; q += al256(2 * rows * 4);
  *spill_keys = (uint64_t*)q; q += al256(n * 8);
  *spill_file = (uint32_t*)q;
}

hipError_t region_group_min(const uint64_t* rkeys, const uint32_t* rfile, uint32_t* cursor,
                            uint64_t cap, uint32_t* out, uint64_t* d_objects, uint64_t* gkeys,
                            uint32_t* gvals, const uint64_t* keys, uint64_t n,
                            const uint64_t* spill_keys, const uint32_t* spill_file,
                            uint32_t fill_limit, hipStream_t s) {
  sd_bucket_min_regions<<<REGIONS, REG_THREADS, 0, s>>>(rkeys, rfile, cursor, cap, out,
                                                        (unsigned long long*)d_objects, gkeys, gvals,
                                                        keys, n, spill_keys, spill_file, fill_limit);
  return hipGetLastError();
}

struct PartPlan {
  uint32_t nb, nblk;
  uint64_t per_block;
};

// blocks: whole PART_TILE trips, at most ~1024 blocks (4 per CU) and nb x blocks <= 2M
// (each block adds its nb counts to the totals with atomics)
static PartPlan part_plan(uint64_t n, uint32_t nb) {
  PartPlan p{nb, 1, PART_TILE};
  const uint64_t trips = n ? (n + PART_TILE - 1) / PART_TILE : 1;
  uint64_t maxblk = MAX_TABLE_ENTRIES / nb;
  if (maxblk > 1024) maxblk = 1024;
  if (maxblk < 1) maxblk = 1;
  const uint64_t nblk = trips < maxblk ? trips : maxblk;
  const uint64_t per = (trips + nblk - 1) / nblk;  // trips per block
  p.per_block = per * PART_TILE;
  p.nblk = (uint32_t)((n + p.per_block - 1) / p.per_block);
  if (p.nblk == 0) p.nblk = 1;
  return p;
}

// Grouping plan: 2^B final buckets of ~TARGET_PER_BUCKET keys, B = b1 + b2 with a coarse
// first level of at most 2^8 buckets (long coalesced runs per block) and a refine level.
struct GroupPlan {
  PartPlan l1;
  uint32_t b1, b2;
  bool big;  // coarse buckets straight to sd_bucket_min_big (no refine level)
  uint32_t nb() const { return 1u << (b1 + b2); }
};

static GroupPlan group_plan(uint64_t n, uint64_t target) {
  if (target == 0) target = TARGET_PER_BUCKET;
  uint32_t bits = 1;
  while (bits < MAX_BITS && ((uint64_t)1 << bits) * target < n) ++bits;
  GroupPlan g;
  // coarse level: 2^8 buckets (runs of ~16 keys per 4,096-key trip); above COARSE10_KEYS,
  // 2^10 (one refine workgroup per coarse bucket walks ~100 K keys instead of ~400 K at 100 M
  // keys: 2.96 -> 2.89 ms; at 12.5 M the 1,024-bucket scatter's shorter runs cost more than
  // the refine saves, 0.307 -> 0.327 ms, profiles/r03b_group_ab/README.md abg5); more only when the
  // refine level would exceed 2^MAX_B2 fine buckets per coarse bucket (> ~200M keys);
  // b1 <= 10 whatever n (MAX_BITS - MAX_B2)
  const uint32_t cb = n <= COARSE10_KEYS ? 8u : 10u;
  g.b1 = bits < cb ? bits : (bits - cb > MAX_B2 ? bits - MAX_B2 : cb);
  g.b2 = bits - g.b1;
  g.big = g.b2 > 0 && n <= BIG_MAX_KEYS;
  if (g.big) g.b2 = 0;
  g.l1 = part_plan(n, 1u << g.b1);
  return g;
}

bool hash_group_supported(uint64_t n) {
  // <= 2^19 buckets at <= 2,500 distinct keys each on average (table fill 3,584): 1.31 G
  return n < (1ull << 32) && n <= ((uint64_t)1 << MAX_BITS) * MAX_MEAN_PER_BUCKET;
}

static uint32_t totals_repl(uint32_t nb) { return nb <= STAGED_MAX_NB ? TOTALS_REPL : 1; }

// The small-batch region chain (sd_region_partition + sd_bucket_min_regions_keys) serves the
// default plan's batches of (SD_SMALL_REGIONS_MIN, BIG_MAX_KEYS] keys: every one (two launches
// against totals + scatter + tables: 20 K keys 0.0219 -> 0.0177 ms, 393 K 0.0260 -> 0.0217,
// 1.31 M 0.0392 -> 0.0314, profiles/r03b_group_ab/README.md "small")
#ifndef SD_SMALL_REGIONS
#define SD_SMALL_REGIONS 1
#endif
#ifndef SD_SMALL_REGIONS_MIN
#define SD_SMALL_REGIONS_MIN 0
#endif
static bool small_regions(uint64_t n, uint64_t target) {
  return SD_SMALL_REGIONS && target == 0 && n > SD_SMALL_REGIONS_MIN && n <= BIG_MAX_KEYS;
}

// the region chain above 1.44 M keys: the default plan's two-level shapes
#ifndef SD_BIG_REGIONS
#define SD_BIG_REGIONS 1
#endif
static uint64_t region_capacity_nb(uint64_t n, uint32_t nb) {
  const double mean = (double)n / nb;
  const double var = mean * (1.0 - 1.0 / nb);
  uint64_t sd = 1;
  while ((double)(sd * sd) < var) ++sd;
  return (uint64_t)mean + 1 + 8 * sd + 64;
}

// its workspace: rkeys | rfile | overflow tables (2n slots) | carve cursor | spill list (n rows)
static size_t small_regions_bytes(uint64_t n) {
  const uint64_t rows = (uint64_t)REGIONS * region_capacity(n);
  return al256(rows * 8) + al256(rows * 4) + al256(2 * n * 8) + al256(2 * n * 4) + 256 +
         al256(n * 8) + al256(n * 4);
}

static bool big_regions(const GroupPlan& g, uint64_t target) {
  return SD_BIG_REGIONS && target == 0 && !g.big && g.b2 > 0 && g.l1.nb <= RBIG_MAX_NB;
}

// rkeys | rfile | spill keys | spill rows | k2 | p2 | starts | Object-count shards | overflow
// tables (2n slots)
static size_t big_regions_bytes(uint64_t n, const GroupPlan& g) {
  const uint64_t rows = (uint64_t)g.l1.nb * region_capacity_nb(n, g.l1.nb);
  return al256(rows * 8) + al256(rows * 4) + 2 * (al256(n * 8) + al256(n * 4)) +
         al256((size_t)g.nb() * 4) + al256(OBJ_SHARDS * OBJ_STRIDE * 8) + al256(2 * n * 8) +
         al256(2 * n * 4);
}

// workspace: k1 | p1 | k2 | p2 | fill (repl copies) | starts1 | starts | Object-count shards |
// overflow tables (the bucket totals live in a persistent buffer of the caller,
// GROUP_TOTALS_WORDS)
size_t hash_group_workspace_bytes(uint64_t n, uint64_t target) {
  const GroupPlan g = group_plan(n, target);
  const size_t nb1 = g.l1.nb;
  const size_t chain = 2 * (al256(n * 8) + al256(n * 4)) + al256(totals_repl(nb1) * nb1 * 4) +
                       al256(nb1 * 4) + al256((size_t)g.nb() * 4) +
                       al256(OBJ_SHARDS * OBJ_STRIDE * 8) + al256(2 * n * 8) + al256(2 * n * 4);
  if (small_regions(n, target)) return std::max(chain, small_regions_bytes(n));
  if (big_regions(g, target)) return std::max(chain, big_regions_bytes(n, g));
  return chain;
}

size_t partition_workspace_bytes(uint64_t n, uint32_t parts) {
  (void)n;
  return 2 * al256((size_t)totals_repl(parts) * parts * 4);
}

// the Object count of a sharded chain: *objects = the sum of its shards
extern "C" __global__ void __launch_bounds__(64)
sd_objects_sum(const unsigned long long* __restrict__ shards, uint32_t nshards,
               unsigned long long* __restrict__ objects) {
  unsigned long long x = threadIdx.x < nshards ? shards[threadIdx.x * OBJ_STRIDE] : 0ull;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, 64);
  if (threadIdx.x == 0) *objects = x;
}

// Zeroes the bucket totals ahead of the chain: a kernel of our own, because a
// hipMemsetAsync fill is a runtime blit whose launch left a ~4 us gap before the next
// kernel (1.31M-key chain: fill 1.8 us + gap 3.8 us of 49 us, profiles/r02b_group_chain_trace.txt)
extern "C" __global__ void __launch_bounds__(256)
sd_zero_words(uint32_t* __restrict__ p, uint32_t n) {
  for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) p[i] = 0;
}

#if SD_DBG
// conservation of the coarse scatter: every (totals replica, bucket) sub-run was reserved
// exactly as far as it was counted (rows reserved == rows counted == rows written)
extern "C" __global__ void __launch_bounds__(256)
sd_dbg_fill_check(const uint32_t* __restrict__ totals, const uint32_t* __restrict__ fill, uint32_t n) {
  for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256)
    SD_DBG_CHECK(fill[i] == totals[i], "scatter sub-run %u: reserved %u, counted %u", i, fill[i],
                 totals[i]);
}
SD_DBG_ACCESSOR(sd_dbg_violations_group_hash)
#endif

// totals (zeroed here unless the caller guarantees them zero) -> bucket-contiguous
// (out_keys, out_pos); starts_out / counts_out
static hipError_t run_partition(const uint64_t* keys, uint64_t n, const PartPlan& p, int mode,
                                uint64_t* out_keys, uint32_t* out_pos, uint32_t* totals,
                                bool totals_zero, uint32_t* fill, uint32_t* starts_out,
                                uint64_t* counts_out, unsigned long long* objects, uint32_t nobj,
                                hipStream_t s,
                                const uint32_t* vals = nullptr, uint32_t* prefill = nullptr) {
  const uint32_t repl = totals_repl(p.nb);
  const uint32_t words = repl * p.nb;
  if (!totals_zero)
    sd_zero_words<<<(words + 255) / 256 < 64 ? (words + 255) / 256 : 64, 256, 0, s>>>(totals, words);
  const size_t lds = (size_t)p.nb * 4, slds = scatter_lds_bytes(p.nb);
  if (mode == 0) {
    if (vals)
      sd_part_totals_mix_vals<<<p.nblk, PART_THREADS, lds, s>>>(keys, n, p.nb, p.per_block, totals, repl,
                                                                fill, objects, nobj, vals, prefill);
    else
      sd_part_totals_mix<<<p.nblk, PART_THREADS, lds, s>>>(keys, n, p.nb, p.per_block, totals, repl,
                                                           fill, objects, nobj, vals, prefill);
    if (p.nb >= 1024)
      sd_part_scatter_mix_wide<<<p.nblk, PART_THREADS, slds, s>>>(keys, n, p.nb, p.per_block, totals, repl,
                                                                  fill, out_keys, out_pos, starts_out);
    else
      sd_part_scatter_mix<<<p.nblk, PART_THREADS, slds, s>>>(keys, n, p.nb, p.per_block, totals, repl,
                                                             fill, out_keys, out_pos, starts_out);
  } else {
    sd_part_totals_range<<<p.nblk, PART_THREADS, lds, s>>>(keys, n, p.nb, p.per_block, totals, repl,
                                                           fill);
    sd_part_scatter_range<<<p.nblk, PART_THREADS, slds, s>>>(keys, n, p.nb, p.per_block, totals,
                                                             repl, fill, out_keys, out_pos, counts_out);
  }
#if SD_DBG
  sd_dbg_fill_check<<<(words + 255) / 256, 256, 0, s>>>(totals, fill, words);
#endif
  return hipGetLastError();
}

// `totals` = the caller's persistent GROUP_TOTALS_WORDS buffer, zero on entry and left zero
// by the chain's last kernel (the bucket tables zero it once the scatter has read it): the
// chain needs no zeroing launch of its own (one dependent launch fewer: 1.31M keys ~0.052 ->
// ~0.048 ms back to back)
hipError_t hash_group_min(const uint64_t* keys, const uint32_t* vals, uint64_t n, uint32_t* out,
                          uint64_t* d_objects, void* ws, uint32_t* totals, hipStream_t s,
                          uint64_t target) {
  if (n == 0) return hipMemsetAsync(d_objects, 0, 8, s);
  if (!hash_group_supported(n)) return hipErrorInvalidValue;
  static_assert(REGIONS * CURSOR_STRIDE + 3 <= GROUP_TOTALS_WORDS,
                "the cursors, spill and done counts fit the totals buffer");
  static_assert((1024 + 1) * CURSOR_STRIDE <= GROUP_TOTALS_WORDS,
                "the big chain's cursors and spill count fit the totals buffer");
  if (small_regions(n, target)) {  // `totals` (zero, left zero) holds the region cursors
    const uint64_t cap = region_capacity(n), rows = (uint64_t)REGIONS * cap;
    char* q = (char*)ws;
    uint64_t* rkeys = (uint64_t*)q; q += al256(rows * 8);
    uint32_t* rfile = (uint32_t*)q; q += al256(rows * 4);
    uint64_t* gkeys = (uint64_t*)q; q += al256(2 * n * 8);
    uint32_t* gvals = (uint32_t*)q; q += al256(2 * n * 4);
    unsigned long long* spill = (unsigned long long*)q; q += 256;
    uint64_t* skeys = (uint64_t*)q; q += al256(n * 8);
    uint32_t* sfile = (uint32_t*)q;
    unsigned long long* obj = (unsigned long long*)d_objects;
    sd_region_partition<<<(uint32_t)((n + RPART_TILE - 1) / RPART_TILE), RPART_THREADS, 0, s>>>(
        keys, vals, n, rkeys, rfile, totals, cap, out, obj, spill, skeys, sfile);
    sd_bucket_min_regions_keys<<<REGIONS, REG_THREADS, 0, s>>>(rkeys, rfile, totals, cap, keys, vals,
                                                               n, out, obj, gkeys, gvals, spill, skeys,
                                                               sfile);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) (void)hipMemsetAsync(totals, 0, GROUP_TOTALS_WORDS * 4, s);  // restore
    return e;
  }
  const GroupPlan g = group_plan(n, target);
  const size_t nb1 = g.l1.nb;
  if (big_regions(g, target)) {  // `totals` (zero, left zero) holds the cursors + spill count
    const uint64_t cap = region_capacity_nb(n, (uint32_t)nb1), rows = nb1 * cap;
    char* q = (char*)ws;
    uint64_t* rkeys = (uint64_t*)q; q += al256(rows * 8);
    uint32_t* rfile = (uint32_t*)q; q += al256(rows * 4);
    uint64_t* skeys = (uint64_t*)q; q += al256(n * 8);
    uint32_t* spos = (uint32_t*)q; q += al256(n * 4);
    uint64_t* k2 = (uint64_t*)q; q += al256(n * 8);
    uint32_t* p2 = (uint32_t*)q; q += al256(n * 4);
    uint32_t* starts = (uint32_t*)q; q += al256((size_t)g.nb() * 4);
    unsigned long long* shards = (unsigned long long*)q; q += al256(OBJ_SHARDS * OBJ_STRIDE * 8);
    uint64_t* gkeys = (uint64_t*)q; q += al256(2 * n * 8);
    uint32_t* gvals = (uint32_t*)q;
    uint32_t* spill_cnt = totals + nb1 * CURSOR_STRIDE;
    const uint32_t twords = (uint32_t)(nb1 * CURSOR_STRIDE + CURSOR_STRIDE);
    const uint64_t tiles = (n + RBIG_TILE - 1) / RBIG_TILE;
    // (8,192-key tiles: 512 x 8 and 256 x 8 were slower, a resident grid prefetching the next
    // tile and 16,384-key tiles staged in two passes no faster: profiles/r03b_group_ab/README.md
    // "big"; the two-pass variant was removed in round 4)
    sd_region_partition_big<<<(uint32_t)tiles, RBIG_THREADS, 0, s>>>(
        keys, vals, n, g.b1, rkeys, rfile, totals, cap, out, shards, OBJ_SHARDS, spill_cnt, skeys, spos);
    sd_part_refine_regions<<<(uint32_t)nb1, PART_THREADS, 0, s>>>(rkeys, rfile, totals, cap, g.b1, g.b2,
                                                                  spill_cnt, skeys, spos, k2, p2, starts);
    sd_bucket_min<<<g.nb(), MIN_THREADS, 0, s>>>(k2, p2, vals, starts, g.nb(), g.b1 + g.b2, n, out,
                                                 shards, gkeys, gvals, totals, twords);
    sd_objects_sum<<<1, 64, 0, s>>>(shards, OBJ_SHARDS, (unsigned long long*)d_objects);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) (void)hipMemsetAsync(totals, 0, GROUP_TOTALS_WORDS * 4, s);  // restore
    return e;
  }
  char* q = (char*)ws;
  uint64_t* k1 = (uint64_t*)q; q += al256(n * 8);
  uint32_t* p1 = (uint32_t*)q; q += al256(n * 4);
  uint64_t* k2 = (uint64_t*)q; q += al256(n * 8);
  uint32_t* p2 = (uint32_t*)q; q += al256(n * 4);
  uint32_t* fill = (uint32_t*)q; q += al256(totals_repl(nb1) * nb1 * 4);
  uint32_t* starts1 = (uint32_t*)q; q += al256(nb1 * 4);
  uint32_t* starts = (uint32_t*)q; q += al256((size_t)g.nb() * 4);
  unsigned long long* shards = (unsigned long long*)q; q += al256(OBJ_SHARDS * OBJ_STRIDE * 8);
  uint64_t* gkeys = (uint64_t*)q; q += al256(2 * n * 8);
  uint32_t* gvals = (uint32_t*)q;
  const uint32_t twords = totals_repl((uint32_t)nb1) * (uint32_t)nb1;  // <= GROUP_TOTALS_WORDS
  // the fine-bucket tables count into the shards (summed after them); the big tables (<= 256
  // workgroups) straight into d_objects
  const bool sharded = !g.big && OBJ_SHARDS > 1;
  unsigned long long* objects = sharded ? shards : (unsigned long long*)d_objects;
  hipError_t e = run_partition(keys, n, g.l1, 0, k1, p1, totals, true, fill, starts1, nullptr,
                               objects, sharded ? OBJ_SHARDS : 1, s, vals, out);
  if (e != hipSuccess) {
    (void)hipMemsetAsync(totals, 0, GROUP_TOTALS_WORDS * 4, s);  // restore the invariant
    return e;
  }
  const uint64_t* fk = k1;
  const uint32_t* fp = p1;
  const uint32_t* fstarts = starts1;
  if (g.b2 > 0) {
    sd_part_refine<<<(uint32_t)nb1, PART_THREADS, 0, s>>>(k1, p1, starts1, (uint32_t)nb1, n, g.b1,
                                                          g.b2, k2, p2, starts);
    fk = k2;
    fp = p2;
    fstarts = starts;
  }
  // (above 1.44M keys, refining into these big tables instead — 4,096 buckets of ~3,050 at
  // 12.5M — was 1.13x slower: profiles/r02b_group_big_tables_ab.log)
  if (g.big)
    sd_bucket_min_big<<<g.nb(), BIG_THREADS, 0, s>>>(fk, fp, vals, fstarts, g.nb(), g.b1, n, out,
                                                     (unsigned long long*)d_objects, gkeys, gvals,
                                                     totals, twords);
  else
    // one workgroup per fine bucket: a persistent grid walking the buckets (with or without
    // the next bucket's first trip prefetched) was 2-10 % slower
    // (profiles/r02b_bucket_min_persist_ab.log)
    // (2,048-slot tables in 256-lane workgroups, twice the buckets: 1.28x slower,
    // profiles/r02b_group_small_tables_ab.log)
  {
    sd_bucket_min<<<g.nb(), MIN_THREADS, 0, s>>>(fk, fp, vals, fstarts, g.nb(), g.b1 + g.b2, n, out,
                                                 objects, gkeys, gvals, totals, twords);
    if (sharded) sd_objects_sum<<<1, 64, 0, s>>>(shards, OBJ_SHARDS, (unsigned long long*)d_objects);
  }
  e = hipGetLastError();
  if (e != hipSuccess) (void)hipMemsetAsync(totals, 0, GROUP_TOTALS_WORDS * 4, s);  // restore
  return e;
}

hipError_t partition_range(const uint64_t* keys, uint64_t n, uint32_t parts, uint64_t* out_keys,
                           uint32_t* out_pos, uint64_t* d_counts, void* ws, hipStream_t s) {
  if (parts == 0 || parts > MAX_BUCKETS || n >= (1ull << 32)) return hipErrorInvalidValue;
  if (n == 0) return hipMemsetAsync(d_counts, 0, (size_t)parts * 8, s);
  const PartPlan p = part_plan(n, parts);
  uint32_t* totals = (uint32_t*)ws;
  uint32_t* fill = (uint32_t*)((char*)ws + al256((size_t)totals_repl(parts) * parts * 4));
  return run_partition(keys, n, p, 1, out_keys, out_pos, totals, false, fill, nullptr, d_counts,
                       nullptr, 0, s);
}

}  // namespace sdcas
