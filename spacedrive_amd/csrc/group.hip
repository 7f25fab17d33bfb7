// group.hip — Object grouping on gfx950: LSD radix sort of (cas key, file idx) pairs and
// segmented run-length grouping (K4 + K5).
//
// Replaces the grouping logic of core/src/object/file_identifier/mod.rs:98-350
// (unique_cas_ids HashSet :149-154, the SQL `cas_id IN (...)` lookup :181-198, the
// linear `find` over existing Objects :214-224, one new Object per remaining file
// :246-311).  Canonical contract: rep(f) = min{ g : key(g) == key(f) },
// objects = #distinct keys.  LSD radix sort is stable and the values enter in ascending
// idx order, so the head of every equal-key run carries the minimum idx.
//
// Sort pass = upsweep (per-tile digit counts in LDS, tile-major, plus per-block sums) ->
// per-digit scan of the block sums -> scatter (stable wave-private ranking with
// 8 ballots per item, the tile staged in LDS in digit order, runs written out coalesced).
// All integer/byte work bound by HBM; nothing here is reshaped into a GEMM.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "sd_debug.h"
#include "sd_group.h"

namespace sdcas {

constexpr int RADIX = 256;
constexpr int SORT_THREADS = 256;
constexpr int SORT_ROUNDS = 16;  // items per thread per tile
constexpr int TILE = SORT_THREADS * SORT_ROUNDS;  // 4096 keys per tile

__device__ __forceinline__ uint32_t digit_of(uint64_t k, uint32_t shift, uint32_t mask) {
  return (uint32_t)(k >> shift) & mask;
}

// Digit counts, tile-major: hist[tile * RADIX + d] = #keys of `tile` with digit d (one
// coalesced 1-KB row per tile; a digit-major store was 256 sectors per tile), and per BLOCK of
// UP_TILES tiles bsum[blk * RADIX + d] = the block's count.  One 256-thread group per tile (a
// block's tiles are counted side by side: as many waves in flight as one workgroup per tile);
// each tile's keys are loaded before its first count (16 loads in flight per lane); each wave
// counts into its own LDS row.
constexpr int UP_TILES = 4;
constexpr int UP_THREADS = UP_TILES * SORT_THREADS;
extern "C" __global__ void __launch_bounds__(UP_THREADS)
sd_radix_upsweep(const uint64_t* __restrict__ keys, uint64_t n, uint32_t shift, uint32_t mask,
                 uint32_t* __restrict__ hist, uint32_t* __restrict__ bsum, uint32_t ntiles) {
  constexpr int WAVES = UP_THREADS / 64;
  __shared__ uint32_t cnt[WAVES][RADIX];
  __shared__ uint32_t tcount[UP_TILES][RADIX];
  const uint32_t t = threadIdx.x, w = t >> 6, g = t / SORT_THREADS, d = t % SORT_THREADS;
  const uint32_t tile = blockIdx.x * UP_TILES + g;
  const uint64_t base = (uint64_t)tile * TILE;
  uint64_t kr[SORT_ROUNDS];
#pragma unroll
  for (int r = 0; r < SORT_ROUNDS; ++r) {
    const uint64_t i = base + (uint64_t)r * SORT_THREADS + d;
    kr[r] = i < n ? keys[i] : 0ull;
  }
#pragma unroll
  for (int v = 0; v < SORT_THREADS / 64; ++v) cnt[g * (SORT_THREADS / 64) + v][d] = 0;
  __syncthreads();
#pragma unroll
  for (int r = 0; r < SORT_ROUNDS; ++r) {
    const uint64_t i = base + (uint64_t)r * SORT_THREADS + d;
    if (i < n) atomicAdd(&cnt[w][digit_of(kr[r], shift, mask)], 1u);
  }
  __syncthreads();
  uint32_t x = 0;
#pragma unroll
  for (int v = 0; v < SORT_THREADS / 64; ++v) x += cnt[g * (SORT_THREADS / 64) + v][d];
  if (tile < ntiles) hist[(uint64_t)tile * RADIX + d] = x;
  tcount[g][d] = x;
  __syncthreads();
  if (g == 0) {
    uint32_t tot = 0;
#pragma unroll
    for (int k = 0; k < UP_TILES; ++k) tot += tcount[k][d];
    bsum[(uint64_t)blockIdx.x * RADIX + d] = tot;
  }
}

// Exclusive scan of the block counts per digit, in place: bsum[b * RADIX + d] = digit d's
// keys in blocks before b; rowtot[d] = digit d's total.  Workgroup g owns digits
// [32g, 32g + 32), thread (seg, d) the seg-th of 32 contiguous block ranges of digit d: it sums
// its range (loads independent, 128 B per row per wave), one LDS scan over the 32 ranges,
// then it rewrites its range as running prefixes.  (The digit bases, the exclusive scan of
// rowtot over 256 digits, are taken by each scatter workgroup itself.)
constexpr int BSCAN_DIGITS = 32, BSCAN_SEGS = 32;
extern "C" __global__ void __launch_bounds__(BSCAN_DIGITS * BSCAN_SEGS)
sd_radix_blockscan(uint32_t* __restrict__ bsum, uint32_t nblk, uint32_t* __restrict__ rowtot) {
  __shared__ uint32_t part[BSCAN_SEGS][BSCAN_DIGITS + 1];
  const uint32_t dsub = threadIdx.x % BSCAN_DIGITS, seg = threadIdx.x / BSCAN_DIGITS;
  const uint32_t d = blockIdx.x * BSCAN_DIGITS + dsub;
  const uint32_t per = (nblk + BSCAN_SEGS - 1) / BSCAN_SEGS;
  const uint32_t b0 = seg * per, b1 = min(nblk, b0 + per);
  uint32_t s = 0;
  for (uint32_t b = b0; b < b1; b += 8) {
    uint32_t x[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) x[k] = b + k < b1 ? bsum[(uint64_t)(b + k) * RADIX + d] : 0u;
#pragma unroll
    for (int k = 0; k < 8; ++k) s += x[k];
  }
  part[seg][dsub] = s;
  __syncthreads();
  uint32_t run = 0, tot = 0;
  for (uint32_t k = 0; k < (uint32_t)BSCAN_SEGS; ++k) {
    const uint32_t x = part[k][dsub];
    if (k < seg) run += x;
    tot += x;
  }
  // rewrite in batches: 8 independent loads, then their 8 stores
  for (uint32_t b = b0; b < b1; b += 8) {
    uint32_t x[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) x[k] = b + k < b1 ? bsum[(uint64_t)(b + k) * RADIX + d] : 0u;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      if (b + k < b1) bsum[(uint64_t)(b + k) * RADIX + d] = run;
      run += x[k];
    }
  }
  if (seg == 0) rowtot[d] = tot;
}

// Stable scatter of one tile, wave-private ranking (round 5).  Wave w owns the contiguous
// quarter [w*1024, (w+1)*1024) of the tile, round r its 64 items from w*1024 + r*64, so the
// tile order (w, r, lane) is the input order and a wave can rank its own items across its
// 16 rounds with no workgroup barrier: wrun[w][d] counts digit d among the wave's earlier
// rounds (only wave w touches row w; one wave's LDS operations complete in program order).
// One barrier then turns the four rows into tile slots: slot = tstart[d] + (digit d in
// earlier waves) + the item's wave-local rank.  3 barriers per tile instead of 33, and 52.7 KB
// of LDS instead of 59 (3 workgroups per CU instead of 2).
// Workgroups are dispatched to the 8 XCDs round-robin (workgroup b on XCD b % 8), and each
// XCD has its own L2.  Tile t's digit-d run ends where tile t+1's begins, so when consecutive
// tiles run on different XCDs the partial 32-B sectors at every run end are written back from
// two L2s (PMC round 5: 219 B/key of scatter traffic for 192).  Round 6: workgroup b takes
// tile xcd_tile(b) — XCD x holds the contiguous tile range [x*q + min(x, r), ...) — so the
// neighbouring runs of the tiles an XCD runs side by side meet in ONE L2.  A permutation of
// the tiles: the result does not depend on it.
constexpr uint32_t XCDS = 8;
__device__ __forceinline__ uint32_t xcd_tile(uint32_t b, uint32_t nt) {
  const uint32_t q = nt / XCDS, r = nt % XCDS, x = b % XCDS;
  return x * q + min(x, r) + b / XCDS;
}

template <bool HAS_VALS>
__device__ __forceinline__ void scatter_body(const uint64_t* __restrict__ keys_in,
                                             const uint32_t* __restrict__ vals_in,
                                             uint64_t* __restrict__ keys_out,
                                             uint32_t* __restrict__ vals_out, uint64_t n,
                                             uint32_t shift, uint32_t mask,
                                             const uint32_t* __restrict__ hist,
                                             const uint32_t* __restrict__ bsum,
                                             const uint32_t* __restrict__ rowtot,
                                             uint32_t ntiles, uint32_t* __restrict__ iota_out) {
  constexpr int WAVES = SORT_THREADS / 64;
  constexpr int WAVE_ITEMS = 64 * SORT_ROUNDS;
  __shared__ uint64_t skey[TILE];
  __shared__ uint32_t sval[TILE];
  __shared__ uint16_t wrun[WAVES][RADIX];  // wave-local digit counts, then wave slot bases
  __shared__ uint32_t gbase[RADIX];
  __shared__ uint16_t tstart[RADIX];
  __shared__ uint32_t wsum[WAVES];
  const uint32_t t = threadIdx.x, lane = t & 63u, w = t >> 6;
  const uint32_t tile = xcd_tile(blockIdx.x, ntiles);
  // digit t's keys in earlier tiles: earlier blocks (scanned) + this block's earlier tiles
  const uint32_t blk = tile / UP_TILES;
  uint32_t mine = bsum[(uint64_t)blk * RADIX + t];
  for (uint32_t tt = blk * UP_TILES; tt < tile; ++tt) mine += hist[(uint64_t)tt * RADIX + t];
  const uint32_t rtot = rowtot[t];
  const uint64_t base = (uint64_t)tile * TILE;
  const uint64_t wbase = base + (uint64_t)w * WAVE_ITEMS;
  uint64_t kr[SORT_ROUNDS];
  uint32_t vr[SORT_ROUNDS];
#pragma unroll
  for (int r = 0; r < SORT_ROUNDS; ++r) {
    const uint64_t i = wbase + (uint64_t)r * 64 + lane;
    kr[r] = i < n ? keys_in[i] : 0ull;
    vr[r] = (HAS_VALS && i < n) ? vals_in[i] : (uint32_t)i;
    // (the first pass of an iota sort can also lay down rep[i] = i for the runs kernel)
    if (!HAS_VALS && iota_out && i < n) iota_out[i] = (uint32_t)i;
  }
#pragma unroll
  for (int j = 0; j < RADIX / 64; ++j) wrun[w][lane + 64 * j] = 0;
  {  // digit base = exclusive scan of the row totals over the 256 digits
    uint32_t inc = rtot;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = __shfl_up(inc, o, 64);
      if (lane >= (uint32_t)o) inc += y;
    }
    if (lane == 63) wsum[w] = inc;
    __syncthreads();
    uint32_t pre = 0;
    for (uint32_t i = 0; i < w; ++i) pre += wsum[i];
    gbase[t] = pre + inc - rtot + mine;
  }
  const uint64_t lt_mask = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  uint32_t dr[SORT_ROUNDS];  // digit << 16 | wave-local rank
#pragma unroll
  for (int r = 0; r < SORT_ROUNDS; ++r) {
    const uint64_t i = wbase + (uint64_t)r * 64 + lane;
    const bool valid = i < n;
    const uint32_t d = digit_of(kr[r], shift, mask);
    uint64_t peers = __ballot(valid);
#pragma unroll
    for (int b = 0; b < 8; ++b) {
      const uint64_t bal = __ballot((d >> b) & 1u);
      peers &= ((d >> b) & 1u) ? bal : ~bal;
    }
    const uint32_t before = valid ? (uint32_t)wrun[w][d] : 0u;
    const uint32_t rank = __popcll(peers & lt_mask);
    dr[r] = (d << 16) | (before + rank);
    if (valid && rank == 0) wrun[w][d] = (uint16_t)(before + __popcll(peers));
  }
  __syncthreads();
  // digit t: tile count, tile start (block exclusive scan), wave slot bases
  uint32_t c[WAVES], cnt = 0;
#pragma unroll
  for (int v = 0; v < WAVES; ++v) { c[v] = wrun[v][t]; cnt += c[v]; }
  uint32_t inc = cnt;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(inc, o, 64);
    if (lane >= (uint32_t)o) inc += y;
  }
  if (lane == 63) wsum[w] = inc;
  // conservation: the wave counts of digit t add up to the upsweep's count of it
  SD_DBG_CHECK(cnt == hist[(uint64_t)tile * RADIX + t], "scatter tile %u digit %u: ranked %u",
               tile, t, cnt);
  __syncthreads();
  uint32_t pre = 0;
  for (uint32_t i = 0; i < w; ++i) pre += wsum[i];
  const uint32_t ts = pre + inc - cnt;
  tstart[t] = (uint16_t)ts;
  uint32_t run = ts;
#pragma unroll
  for (int v = 0; v < WAVES; ++v) { wrun[v][t] = (uint16_t)run; run += c[v]; }
  __syncthreads();
#pragma unroll
  for (int r = 0; r < SORT_ROUNDS; ++r) {
    const uint64_t i = wbase + (uint64_t)r * 64 + lane;
    if (i < n) {
      const uint32_t slot = (uint32_t)wrun[w][dr[r] >> 16] + (dr[r] & 0xFFFFu);
      skey[slot] = kr[r];
      sval[slot] = vr[r];
    }
  }
  __syncthreads();
  const uint32_t tile_n = (uint32_t)(n - base < (uint64_t)TILE ? n - base : (uint64_t)TILE);
  for (uint32_t s = t; s < tile_n; s += SORT_THREADS) {
    const uint64_t k = skey[s];
    const uint32_t d = digit_of(k, shift, mask);
    const uint32_t pos = gbase[d] + (s - tstart[d]);
    keys_out[pos] = k;
    vals_out[pos] = sval[s];
  }
}

extern "C" __global__ void __launch_bounds__(SORT_THREADS)
sd_radix_scatter(const uint64_t* __restrict__ keys_in, const uint32_t* __restrict__ vals_in,
                 uint64_t* __restrict__ keys_out, uint32_t* __restrict__ vals_out, uint64_t n,
                 uint32_t shift, uint32_t mask, const uint32_t* __restrict__ hist,
                 const uint32_t* __restrict__ bsum, const uint32_t* __restrict__ rowtot,
                 uint32_t ntiles) {
  scatter_body<true>(keys_in, vals_in, keys_out, vals_out, n, shift, mask, hist, bsum, rowtot,
                     ntiles, nullptr);
}

extern "C" __global__ void __launch_bounds__(SORT_THREADS)
sd_radix_scatter_iota(const uint64_t* __restrict__ keys_in, uint64_t* __restrict__ keys_out,
                      uint32_t* __restrict__ vals_out, uint64_t n, uint32_t shift, uint32_t mask,
                      const uint32_t* __restrict__ hist, const uint32_t* __restrict__ bsum,
                      const uint32_t* __restrict__ rowtot, uint32_t ntiles,
                      uint32_t* __restrict__ iota_out) {
  scatter_body<false>(keys_in, nullptr, keys_out, vals_out, n, shift, mask, hist, bsum, rowtot,
                      ntiles, iota_out);
}

// ---- device-wide exclusive scan (u32, sum) over m <= SCAN_TILE^2 elements ----------
constexpr int SCAN_THREADS = 256;
constexpr int SCAN_ITEMS = 16;
constexpr int SCAN_TILE = SCAN_THREADS * SCAN_ITEMS;  // 4096

__device__ __forceinline__ uint32_t block_exclusive_sum(uint32_t x, uint32_t* total) {
  __shared__ uint32_t wsum[SCAN_THREADS / 64];
  const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
  uint32_t inc = x;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(inc, o, 64);
    if (lane >= (uint32_t)o) inc += y;
  }
  if (lane == 63) wsum[w] = inc;
  __syncthreads();
  uint32_t wpre = 0, tot = 0;
#pragma unroll
  for (int i = 0; i < SCAN_THREADS / 64; ++i) {
    const uint32_t s = wsum[i];
    if ((uint32_t)i < w) wpre += s;
    tot += s;
  }
  __syncthreads();
  *total = tot;
  return wpre + inc - x;
}

// per-tile sums
extern "C" __global__ void __launch_bounds__(SCAN_THREADS)
sd_scan_reduce(const uint32_t* __restrict__ in, uint64_t m, uint32_t* __restrict__ partial) {
  const uint64_t base = (uint64_t)blockIdx.x * SCAN_TILE + (uint64_t)threadIdx.x * SCAN_ITEMS;
  uint32_t s = 0;
#pragma unroll
  for (int k = 0; k < SCAN_ITEMS; ++k) s += (base + k < m) ? in[base + k] : 0u;
  uint32_t tot;
  (void)block_exclusive_sum(s, &tot);
  if (threadIdx.x == 0) partial[blockIdx.x] = tot;
}

// exclusive scan of a tile (blocked per thread), seeded with tile_offset[blockIdx] (or 0)
extern "C" __global__ void __launch_bounds__(SCAN_THREADS)
sd_scan_tiles(const uint32_t* __restrict__ in, uint64_t m, uint32_t* __restrict__ out,
              const uint32_t* __restrict__ tile_offset) {
  const uint64_t base = (uint64_t)blockIdx.x * SCAN_TILE + (uint64_t)threadIdx.x * SCAN_ITEMS;
  uint32_t v[SCAN_ITEMS];
  uint32_t s = 0;
#pragma unroll
  for (int k = 0; k < SCAN_ITEMS; ++k) { v[k] = (base + k < m) ? in[base + k] : 0u; s += v[k]; }
  uint32_t tot;
  uint32_t run = block_exclusive_sum(s, &tot) + (tile_offset ? tile_offset[blockIdx.x] : 0u);
#pragma unroll
  for (int k = 0; k < SCAN_ITEMS; ++k) {
    if (base + k < m) out[base + k] = run;
    run += v[k];
  }
}

// ---- grouping over the sorted pairs -------------------------------------------------
// Run heads + rep in ONE pass over the sorted pairs (round 6; round 5 ran tile heads -> a
// single-workgroup carry scan -> emit, reading the keys twice and staging 52 KB of LDS per
// workgroup).  Workgroup = one SCAN_TILE of sorted positions, wave w the contiguous quarter
// [w*1024, (w+1)*1024) as 16 rounds of 64 consecutive positions (coalesced loads, all issued
// up front).  A position is a head iff its key differs from its predecessor's (the previous
// lane's by a shuffle, the previous round's last lane, or one load before the wave); a lane's
// run head is the highest head lane at or below it (one ballot + clz), else the last head of
// the wave's earlier rounds (a wave-uniform carry).  No LDS staging and no barrier in the
// rounds; the positions of a wave before its first head (a run entering the wave, usually
// none) are resolved after ONE barrier from the last head of an earlier wave, else from the
// run entering the tile: its head is the key's FIRST position, a lower bound found by wave 0
// galloping back from tile0 - 1 and bisecting (a few dependent loads for the short runs of
// real libraries, ~2 log2(n) for one hot key, one if the key starts at position 0).
// rep[v] = the head's val for every run member; PREFILLED: rep[v] == v already holds for
// every val (the iota sort's first pass wrote it), so only members that are not heads store —
// a library without duplicates writes nothing here.  The tile's head count goes to
// tile_heads[] (the Object total, summed by sd_sum_u32_block).

// first position of key K in the sorted keys, given skeys[hi] == K (hi < 2^32)
__device__ uint32_t run_first(const uint64_t* __restrict__ skeys, uint64_t K, int64_t hi) {
  if (skeys[0] == K) return 0;  // (one key everywhere: one load)
  int64_t lo = 0, step = 1;     // invariant: skeys[lo] < K == skeys[hi]
  for (;;) {
    const int64_t j = hi - step;
    if (j <= 0) break;
    if (skeys[j] != K) { lo = j; break; }
    hi = j;
    step <<= 1;
  }
  while (hi - lo > 1) {
    const int64_t mid = lo + (hi - lo) / 2;
    if (skeys[mid] == K) hi = mid; else lo = mid;
  }
  return (uint32_t)hi;
}

constexpr uint32_t RUN_WAVES = SCAN_THREADS / 64;
constexpr uint32_t RUN_ROUNDS = SCAN_TILE / SCAN_THREADS;  // 16 rounds of 64 per wave

template <bool PREFILLED>
__device__ __forceinline__ void group_runs_body(const uint64_t* __restrict__ skeys,
                                                const uint32_t* __restrict__ svals, uint64_t n,
                                                uint32_t* __restrict__ rep,
                                                uint32_t* __restrict__ tile_heads) {
  __shared__ uint32_t w_val[RUN_WAVES];    // the val of the wave's last head
  __shared__ uint32_t w_has[RUN_WAVES];    // the wave holds a head
  __shared__ uint32_t w_heads[RUN_WAVES];  // heads in the wave
  __shared__ uint32_t tile_carry;          // the val of the head of the run entering the tile
  const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
  const uint64_t tile0 = (uint64_t)blockIdx.x * SCAN_TILE;
  const uint64_t wbase = tile0 + (uint64_t)w * (64 * RUN_ROUNDS);
  uint64_t kr[RUN_ROUNDS];
  uint32_t vr[RUN_ROUNDS];
#pragma unroll
  for (int r = 0; r < (int)RUN_ROUNDS; ++r) {
    const uint64_t i = wbase + (uint64_t)r * 64 + lane;
    kr[r] = i < n ? skeys[i] : 0ull;
    vr[r] = i < n ? svals[i] : 0u;
  }
  // the key before the wave (wave-uniform)
  uint64_t prevk = (wbase > 0 && wbase <= n) ? skeys[wbase - 1] : 0ull;
  uint32_t carry_val = 0, heads = 0, npend = 0;
  bool carry = false;  // a head seen in this wave's earlier rounds
  const uint64_t le_mask = ~0ull >> (63u - lane);  // lanes <= this lane
#pragma unroll
  for (int r = 0; r < (int)RUN_ROUNDS; ++r) {
    const uint64_t i = wbase + (uint64_t)r * 64 + lane;
    const bool valid = i < n;
    uint64_t kp = __shfl_up(kr[r], 1, 64);
    if (lane == 0) kp = prevk;
    const bool head = valid && (i == 0 || kr[r] != kp);
    const uint64_t hmask = __ballot(head);
    const uint64_t mine = hmask & le_mask;
    // the val of this lane's run head: a head lane of this round, else the carried one
    const uint32_t hl = mine ? 63u - (uint32_t)__clzll(mine) : 0u;
    const uint32_t hv = __shfl(vr[r], (int)hl, 64);
    if (valid) {
      if (head) {
        if (!PREFILLED) rep[vr[r]] = vr[r];
      } else if (mine) {
        rep[vr[r]] = hv;
      } else if (carry) {
        rep[vr[r]] = carry_val;
      }  // else: before the wave's first head, resolved below
    }
    if (!carry) npend += (uint32_t)__popcll(__ballot(valid && !mine));
    if (hmask) {
      carry = true;
      carry_val = __shfl(vr[r], 63 - __clzll(hmask), 64);
    }
    heads += (uint32_t)__popcll(hmask);
    prevk = __shfl(kr[r], 63, 64);
  }
  if (lane == 0) {
    w_val[w] = carry_val;
    w_has[w] = carry ? 1u : 0u;
    w_heads[w] = heads;
    // wave 0 before a head: the run entering the tile (its head is before tile0)
    if (w == 0) tile_carry = (npend && tile0 < n) ? svals[run_first(skeys, skeys[tile0], (int64_t)tile0 - 1)] : 0u;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t t = 0;
#pragma unroll
    for (uint32_t k = 0; k < RUN_WAVES; ++k) t += w_heads[k];
    tile_heads[blockIdx.x] = t;
  }
  if (npend) {  // (wave-uniform) positions [wbase, wbase + npend) continue an earlier run
    uint32_t hv = tile_carry;
    for (int k = (int)w - 1; k >= 0; --k)
      if (w_has[k]) { hv = w_val[k]; break; }
    for (uint32_t j = lane; j < npend; j += 64) rep[svals[wbase + j]] = hv;
  }
}

extern "C" __global__ void __launch_bounds__(SCAN_THREADS)
sd_group_runs(const uint64_t* __restrict__ skeys, const uint32_t* __restrict__ svals, uint64_t n,
              uint32_t* __restrict__ rep, uint32_t* __restrict__ tile_heads) {
  group_runs_body<false>(skeys, svals, n, rep, tile_heads);
}
extern "C" __global__ void __launch_bounds__(SCAN_THREADS)
sd_group_runs_prefilled(const uint64_t* __restrict__ skeys, const uint32_t* __restrict__ svals,
                        uint64_t n, uint32_t* __restrict__ rep, uint32_t* __restrict__ tile_heads) {
  group_runs_body<true>(skeys, svals, n, rep, tile_heads);
}

// *total = sum of v[0..m) in u64 (one workgroup; m <= SCAN_TILE tile sums, or one tile):
// callers of a u32 scan whose sum may pass 2^32 check the true total with it
extern "C" __global__ void __launch_bounds__(SCAN_THREADS)
sd_sum_u32_block(const uint32_t* __restrict__ v, uint64_t m, unsigned long long* __restrict__ total) {
  __shared__ unsigned long long red[SCAN_THREADS];
  unsigned long long acc = 0;
  for (uint64_t i = threadIdx.x; i < m; i += SCAN_THREADS) acc += v[i];
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int h = SCAN_THREADS / 2; h > 0; h >>= 1) {
    if ((int)threadIdx.x < h) red[threadIdx.x] += red[threadIdx.x + h];
    __syncthreads();
  }
  if (threadIdx.x == 0) *total = red[0];
}

// chunk-of-`chunk` reference emulation (mod.rs:202-311):
// rep_c[i] = i if canonical rep is in i's own chunk, else canonical rep.  The created count
// is summed per workgroup (CHUNKED_ROWS rows) and added with one device atomic: one per wave
// on one counter serialised (same-address device atomics complete one per ~12.8 ns,
// tools/ubench_bucketload.hip).
constexpr int CHUNKED_THREADS = 1024, CHUNKED_ITEMS = 8;
constexpr uint32_t CHUNKED_ROWS = CHUNKED_THREADS * CHUNKED_ITEMS;
extern "C" __global__ void __launch_bounds__(CHUNKED_THREADS)
sd_group_chunked(const uint32_t* __restrict__ rep, uint64_t n, uint32_t chunk,
                 uint32_t* __restrict__ rep_chunked, unsigned long long* __restrict__ created) {
  __shared__ unsigned int wsum;
  if (threadIdx.x == 0) wsum = 0;
  __syncthreads();
  uint32_t mine = 0;
#pragma unroll
  for (int j = 0; j < CHUNKED_ITEMS; ++j) {
    const uint64_t i = (uint64_t)blockIdx.x * CHUNKED_ROWS + (uint64_t)j * CHUNKED_THREADS + threadIdx.x;
    if (i < n) {
      const uint32_t r = rep[i];
      const bool own = (r / chunk) == ((uint32_t)i / chunk);
      rep_chunked[i] = own ? (uint32_t)i : r;
      mine += own;
    }
  }
  // the wave's sum by ballots of the bits of `mine` (<= CHUNKED_ITEMS < 16)
  const uint32_t wave = __popcll(__ballot(mine & 1u)) + 2u * __popcll(__ballot(mine & 2u)) +
                        4u * __popcll(__ballot(mine & 4u)) + 8u * __popcll(__ballot(mine & 8u));
  if ((threadIdx.x & 63u) == 0 && wave) atomicAdd(&wsum, wave);
  __syncthreads();
  if (threadIdx.x == 0 && wsum) atomicAdd(created, (unsigned long long)wsum);
}

// helpers of group_min_by_sort: widen the values to sort keys, gather keys by position,
// and out[i] = vals[rep[i]]
extern "C" __global__ void __launch_bounds__(256)
sd_widen_vals(const uint32_t* __restrict__ vals, uint64_t n, uint64_t* __restrict__ out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = vals ? vals[i] : (uint32_t)i;
}
extern "C" __global__ void __launch_bounds__(256)
sd_gather_keys(const uint64_t* __restrict__ keys, const uint32_t* __restrict__ idx, uint64_t n,
               uint64_t* __restrict__ out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = keys[idx[i]];
}
extern "C" __global__ void __launch_bounds__(256)
sd_gather_vals(const uint32_t* __restrict__ vals, const uint32_t* __restrict__ rep, uint64_t n,
               uint32_t* __restrict__ out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = vals ? vals[rep[i]] : rep[i];
}

}  // namespace sdcas

// ---- host launchers ----------------------------------------------------------------
namespace sdcas {

SD_DBG_ACCESSOR(sd_dbg_violations_group)

static inline size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }
static inline uint32_t tiles_of(uint64_t n, uint64_t tile) { return (uint32_t)((n + tile - 1) / tile); }

size_t sort_workspace_bytes(uint64_t n) {
  const uint64_t nt = tiles_of(n ? n : 1, TILE);
  const uint64_t nb = tiles_of(nt, UP_TILES);
  return align_up(n * 8, 256) + align_up(n * 4, 256) + align_up(RADIX * nt * 4, 256) +
         align_up(RADIX * nb * 4, 256) + align_up(RADIX * 4, 256) + 256;
}

size_t group_workspace_bytes(uint64_t n) {
  const uint64_t ng = tiles_of(n ? n : 1, SCAN_TILE);
  return sort_workspace_bytes(n) + align_up(n * 8, 256) + align_up(n * 4, 256) +
         3 * align_up(ng * 4, 256) + 256;
}

hipError_t exclusive_scan_u32(const uint32_t* in, uint32_t* out, uint64_t m, uint32_t* partial,
                              hipStream_t s, unsigned long long* total) {
  const uint32_t nt = tiles_of(m, SCAN_TILE);
  if (nt <= 1) {
    if (total) sd_sum_u32_block<<<1, SCAN_THREADS, 0, s>>>(in, m, total);
    sd_scan_tiles<<<1, SCAN_THREADS, 0, s>>>(in, m, out, nullptr);
    return hipGetLastError();
  }
  if (nt > (uint32_t)SCAN_TILE) return hipErrorInvalidValue;
  sd_scan_reduce<<<nt, SCAN_THREADS, 0, s>>>(in, m, partial);
  // the tile sums before their (u32) scan: the true total, even when the scan wraps
  if (total) sd_sum_u32_block<<<1, SCAN_THREADS, 0, s>>>(partial, nt, total);
  sd_scan_tiles<<<1, SCAN_THREADS, 0, s>>>(partial, nt, partial, nullptr);
  sd_scan_tiles<<<nt, SCAN_THREADS, 0, s>>>(in, m, out, partial);
  return hipGetLastError();
}

hipError_t radix_sort_pairs(const uint64_t* keys_in, const uint32_t* vals_in, uint64_t* keys_out,
                            uint32_t* vals_out, uint64_t n, int begin_bit, int end_bit, void* ws,
                            hipStream_t s, uint32_t* iota_out) {
  if (n == 0) return hipSuccess;
  if (n >= (1ull << 32) || begin_bit < 0 || end_bit > 64 || end_bit <= begin_bit)
    return hipErrorInvalidValue;
  const uint32_t nt = tiles_of(n, TILE);
  const uint32_t nb = tiles_of(nt, UP_TILES);
  char* p = (char*)ws;
  uint64_t* kalt = (uint64_t*)p; p += align_up(n * 8, 256);
  uint32_t* valt = (uint32_t*)p; p += align_up(n * 4, 256);
  uint32_t* hist = (uint32_t*)p; p += align_up((uint64_t)RADIX * nt * 4, 256);
  uint32_t* bsum = (uint32_t*)p; p += align_up((uint64_t)RADIX * nb * 4, 256);
  uint32_t* rowtot = (uint32_t*)p;
  const int passes = (end_bit - begin_bit + 7) / 8;
  const uint64_t* ksrc = keys_in;
  const uint32_t* vsrc = vals_in;
  for (int i = 0; i < passes; ++i) {
    const uint32_t shift = (uint32_t)(begin_bit + 8 * i);
    const int bits = (end_bit - (int)shift) < 8 ? (end_bit - (int)shift) : 8;
    const uint32_t mask = (1u << bits) - 1u;
    const bool to_out = ((passes - 1 - i) % 2) == 0;
    uint64_t* kdst = to_out ? keys_out : kalt;
    uint32_t* vdst = to_out ? vals_out : valt;
    sd_radix_upsweep<<<nb, UP_THREADS, 0, s>>>(ksrc, n, shift, mask, hist, bsum, nt);
    sd_radix_blockscan<<<RADIX / BSCAN_DIGITS, BSCAN_DIGITS * BSCAN_SEGS, 0, s>>>(bsum, nb, rowtot);
    if (vsrc)
      sd_radix_scatter<<<nt, SORT_THREADS, 0, s>>>(ksrc, vsrc, kdst, vdst, n, shift, mask, hist, bsum,
                                                   rowtot, nt);
    else
      sd_radix_scatter_iota<<<nt, SORT_THREADS, 0, s>>>(ksrc, kdst, vdst, n, shift, mask, hist, bsum,
                                                        rowtot, nt, iota_out);
    ksrc = kdst;
    vsrc = vdst;
  }
  return hipGetLastError();
}

hipError_t group_sorted(const uint64_t* skeys, const uint32_t* svals, uint64_t n, uint32_t* rep,
                        uint64_t* d_objects, void* ws, hipStream_t s, bool rep_prefilled) {
  if (n == 0) return hipMemsetAsync(d_objects, 0, 8, s);
  const uint32_t ng = tiles_of(n, SCAN_TILE);
  uint32_t* heads = (uint32_t*)ws;
  if (rep_prefilled)
    sd_group_runs_prefilled<<<ng, SCAN_THREADS, 0, s>>>(skeys, svals, n, rep, heads);
  else
    sd_group_runs<<<ng, SCAN_THREADS, 0, s>>>(skeys, svals, n, rep, heads);
  sd_sum_u32_block<<<1, SCAN_THREADS, 0, s>>>(heads, ng, (unsigned long long*)d_objects);
  return hipGetLastError();
}

hipError_t group_keys(const uint64_t* keys, uint64_t n, uint32_t* rep, uint64_t* d_objects,
                      void* ws, hipStream_t s) {
  if (n == 0) return hipMemsetAsync(d_objects, 0, 8, s);
  char* p = (char*)ws;
  char* sort_ws = p; p += sort_workspace_bytes(n);
  uint64_t* skeys = (uint64_t*)p; p += align_up(n * 8, 256);
  uint32_t* svals = (uint32_t*)p; p += align_up(n * 4, 256);
  // (the first pass also writes rep[i] = i: the runs kernel then stores only duplicates)
  hipError_t e = radix_sort_pairs(keys, nullptr, skeys, svals, n, 0, 64, sort_ws, s, rep);
  if (e != hipSuccess) return e;
  return group_sorted(skeys, svals, n, rep, d_objects, p, s, true);
}

size_t group_min_sorted_workspace_bytes(uint64_t n) {
  return group_workspace_bytes(n) + 3 * align_up(n * 8, 256) + 3 * align_up(n * 4, 256) + 256;
}

// out[i] = min{ val(j) : keys[j] == keys[i] } through two stable LSD sorts: positions by
// value (32 bits), then by key (64 bits) — inside every equal-key run the positions ascend
// by value, so the run head holds the minimum (sd_cas_group_min_dev beyond the hash
// grouping's range).
hipError_t group_min_by_sort(const uint64_t* keys, const uint32_t* vals, uint64_t n, uint32_t* out,
                             uint64_t* d_objects, void* ws, hipStream_t s) {
  if (n == 0) return hipMemsetAsync(d_objects, 0, 8, s);
  char* p = (char*)ws;
  char* gws = p; p += group_workspace_bytes(n);
  uint64_t* vkey = (uint64_t*)p; p += align_up(n * 8, 256);
  uint64_t* k2 = (uint64_t*)p; p += align_up(n * 8, 256);
  uint64_t* skeys = (uint64_t*)p; p += align_up(n * 8, 256);
  uint32_t* order = (uint32_t*)p; p += align_up(n * 4, 256);
  uint32_t* spos = (uint32_t*)p; p += align_up(n * 4, 256);
  uint32_t* rep = (uint32_t*)p;
  const uint32_t nb = tiles_of(n, 256);
  sd_widen_vals<<<nb, 256, 0, s>>>(vals, n, vkey);
  // (spos is a permutation of the positions, so rep can be prefilled by the first sort)
  hipError_t e = radix_sort_pairs(vkey, nullptr, k2, order, n, 0, 32, gws, s, rep);
  if (e != hipSuccess) return e;
  sd_gather_keys<<<nb, 256, 0, s>>>(keys, order, n, k2);
  e = radix_sort_pairs(k2, order, skeys, spos, n, 0, 64, gws, s);
  if (e != hipSuccess) return e;
  e = group_sorted(skeys, spos, n, rep, d_objects, gws, s, true);
  if (e != hipSuccess) return e;
  sd_gather_vals<<<nb, 256, 0, s>>>(vals, rep, n, out);
  return hipGetLastError();
}

hipError_t group_chunked(const uint32_t* rep, uint64_t n, uint32_t chunk, uint32_t* rep_chunked,
                         uint64_t* d_created, hipStream_t s) {
  if (n == 0) return hipSuccess;
  if (chunk == 0) return hipErrorInvalidValue;
  sd_group_chunked<<<(uint32_t)((n + CHUNKED_ROWS - 1) / CHUNKED_ROWS), CHUNKED_THREADS, 0, s>>>(rep, n, chunk, rep_chunked,
                                                   (unsigned long long*)d_created);
  return hipGetLastError();
}

}  // namespace sdcas
