// multi.hip — small kernels of the single-process multi-device grouping (sd_cas_multi_*).
//
// The exchange itself is peer copies (hipMemcpyPeerAsync over xGMI) driven by
// sd_hip_cas.cpp; these kernels compute the key-range split points on the sorted keys,
// build global file indices, gather run representatives and scatter them back.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "sd_multi.h"

namespace sdcas {

// splits[r] = #keys < ceil(r * 2^64 / G) for r = 1..G-1 (keys sorted ascending, unsigned);
// splits[0] = 0, splits[G] = n.  One thread per boundary: binary search.
extern "C" __global__ void sd_multi_splits(const uint64_t* __restrict__ skeys, uint64_t n,
                                           uint32_t G, uint64_t* __restrict__ splits) {
  const uint32_t r = threadIdx.x;
  if (r > G) return;
  if (r == 0) { splits[0] = 0; return; }
  if (r == G) { splits[G] = n; return; }
  // boundary b = ceil(r * 2^64 / G) in 64-bit arithmetic: 2^64 = Q*G + R, so
  // r * 2^64 / G = r*Q + r*R/G with r*R < G^2 (G <= 1023)
  const uint64_t q1 = ~0ull / G, r1 = ~0ull % G;  // 2^64 - 1 = q1*G + r1
  const uint64_t Q = (r1 + 1 == G) ? q1 + 1 : q1, R = (r1 + 1 == G) ? 0 : r1 + 1;
  const uint64_t b = (uint64_t)r * Q + ((uint64_t)r * R + G - 1) / G;
  uint64_t lo = 0, hi = n;
  while (lo < hi) {  // first index with key >= b
    const uint64_t mid = (lo + hi) >> 1;
    if (skeys[mid] < b) lo = mid + 1; else hi = mid;
  }
  splits[r] = lo;
}

// ---- the RCCL key-range exchange of spacedrive_amd/shard.py (one process per GPU) ----
// rows[j] = (key lo32, key hi32, u32 global idx file0 + pos[j]): 12-byte rows, one
// all-to-all instead of a key and an idx exchange
extern "C" __global__ void __launch_bounds__(256)
sd_exch_pack(const uint64_t* __restrict__ keys, const uint32_t* __restrict__ pos, uint64_t n,
             uint64_t file0, uint32_t* __restrict__ rows) {
  const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j < n) {
    const uint64_t k = keys[j];
    rows[3 * j] = (uint32_t)k;
    rows[3 * j + 1] = (uint32_t)(k >> 32);
    rows[3 * j + 2] = (uint32_t)(file0 + pos[j]);
  }
}

// received rows -> keys[m] u64 + vals[m] u32 (the grouping's inputs)
extern "C" __global__ void __launch_bounds__(256)
sd_exch_split(const uint32_t* __restrict__ rows, uint64_t m, uint64_t* __restrict__ keys,
              uint32_t* __restrict__ vals) {
  const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j < m) {
    keys[j] = (uint64_t)rows[3 * j] | ((uint64_t)rows[3 * j + 1] << 32);
    vals[j] = rows[3 * j + 2];
  }
}

// rep[pos[j]] = back[j]: the mirrored u32 reps scattered to local file order (as u64)
extern "C" __global__ void __launch_bounds__(256)
sd_exch_unpack(const uint32_t* __restrict__ back, const uint32_t* __restrict__ pos, uint64_t n,
               uint64_t* __restrict__ rep) {
  const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j < n) rep[pos[j]] = back[j];
}

// ---- fixed-capacity exchange (no host round trip for the part sizes) -----------------
// Every rank sends G blocks of `cap` rows (+ G spill blocks of `spill` rows) whatever its
// part sizes are: BLAKE3 keys are uniform, so a part of a rank's n keys is n/G +- a few
// sqrt(n/G) and fits a capacity fixed up front; all_to_all then needs no split lists and
// the step no host sync.  Unused slots carry a sentinel key that lies outside the
// receiver's key range (the first key of the next range), so it never merges with a real
// key; a part larger than cap + spill raises `overflow` (the caller then redoes the step
// with the exact, size-exchanging path).

// first key of range r of G: ceil(r * 2^64 / G) (r = G wraps to 0)
__device__ __forceinline__ uint64_t range_start(uint32_t r, uint32_t G) {
  if (r == 0 || r >= G) return 0;
  const uint64_t q1 = ~0ull / G, r1 = ~0ull % G;  // 2^64 - 1 = q1*G + r1
  const uint64_t Q = (r1 + 1 == G) ? q1 + 1 : q1, R = (r1 + 1 == G) ? 0 : r1 + 1;
  return (uint64_t)r * Q + ((uint64_t)r * R + G - 1) / G;
}

constexpr uint32_t FIXED_MAX_G = 1024;

// Part offsets o_p = sum_{q<p} counts[q] into LDS (G <= FIXED_MAX_G).
__device__ __forceinline__ void part_offsets(const uint64_t* counts, uint32_t G, uint64_t* off) {
  if (threadIdx.x == 0) {
    uint64_t run = 0;
    for (uint32_t p = 0; p < G; ++p) { off[p] = run; run += counts[p]; }
  }
  __syncthreads();
}

extern "C" __global__ void __launch_bounds__(256)
sd_exch_pack_fixed(const uint64_t* __restrict__ keys, const uint32_t* __restrict__ pos,
                   const uint64_t* __restrict__ counts, uint32_t G, uint64_t cap, uint64_t spill,
                   uint64_t file0, uint32_t* __restrict__ rows, uint32_t* __restrict__ srows,
                   uint32_t* __restrict__ overflow) {
  __shared__ uint64_t off[FIXED_MAX_G];
  part_offsets(counts, G, off);
  const uint64_t total = (uint64_t)G * (cap + spill);
  for (uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; s < total;
       s += (uint64_t)gridDim.x * blockDim.x) {
    uint32_t p;
    uint64_t t;
    uint32_t* dst;
    if (s < (uint64_t)G * cap) {
      p = (uint32_t)(s / cap); t = s % cap; dst = rows + 3 * s;
    } else {
      const uint64_t s2 = s - (uint64_t)G * cap;
      p = (uint32_t)(s2 / spill); t = cap + s2 % spill; dst = srows + 3 * s2;
    }
    uint64_t k;
    uint32_t v;
    if (t < counts[p]) {
      const uint64_t j = off[p] + t;
      k = keys[j];
      v = (uint32_t)(file0 + pos[j]);
    } else {
      k = range_start(p + 1, G);  // outside receiver p's range [start(p), start(p+1))
      v = 0xFFFFFFFFu;
    }
    dst[0] = (uint32_t)k;
    dst[1] = (uint32_t)(k >> 32);
    dst[2] = v;
    if (t == cap + spill - 1 && counts[p] > cap + spill) atomicOr(overflow, 1u);
  }
}

// received rows -> keys/vals.  A sentinel row (key == this receiver's sentinel) gets the
// distinct key sentinel + j: still outside the receiver's range (m < 2^64 - range width),
// so it never merges with a real key, and the padding of a step (~8% of the rows) no longer
// forms one hot key whose bucket serialises the grouping (world 8, 1.42 M rows: group_min
// 0.168 -> 0.074 ms, profiles/r02_exchange_timing.log).  sentinel_rows += their number
// (each is one extra Object, subtracted by the caller): counted per workgroup in LDS, one
// device atomic per workgroup that saw any (one per wave put ~1,700 same-address atomics in
// a row: 0.035 ms for the split alone).
constexpr int SPLIT_THREADS = 256, SPLIT_ITEMS = 8;
extern "C" __global__ void __launch_bounds__(SPLIT_THREADS)
sd_exch_split_fixed(const uint32_t* __restrict__ rows, uint64_t m, uint64_t sentinel,
                    uint64_t* __restrict__ keys, uint32_t* __restrict__ vals,
                    unsigned long long* __restrict__ sentinel_rows) {
  __shared__ uint32_t nsent;
  if (threadIdx.x == 0) nsent = 0;
  __syncthreads();
  const uint64_t base = (uint64_t)blockIdx.x * SPLIT_THREADS * SPLIT_ITEMS + threadIdx.x;
  uint32_t lo[SPLIT_ITEMS], hi[SPLIT_ITEMS], v[SPLIT_ITEMS];
#pragma unroll
  for (int i = 0; i < SPLIT_ITEMS; ++i) {
    const uint64_t j = base + (uint64_t)i * SPLIT_THREADS;
    if (j < m) { lo[i] = rows[3 * j]; hi[i] = rows[3 * j + 1]; v[i] = rows[3 * j + 2]; }
  }
  uint32_t hits = 0;
#pragma unroll
  for (int i = 0; i < SPLIT_ITEMS; ++i) {
    const uint64_t j = base + (uint64_t)i * SPLIT_THREADS;
    if (j < m) {
      const uint64_t k = (uint64_t)lo[i] | ((uint64_t)hi[i] << 32);
      const bool hit = k == sentinel;
      hits += hit;
      keys[j] = hit ? sentinel + j : k;
      vals[j] = v[i];
    }
  }
  if (hits) atomicAdd(&nsent, hits);
  __syncthreads();
  if (threadIdx.x == 0 && nsent) atomicAdd(sentinel_rows, (unsigned long long)nsent);
}

// rep[pos[o_p + t]] = back (main block t < cap, spill block otherwise) for t < counts[p]
extern "C" __global__ void __launch_bounds__(256)
sd_exch_unpack_fixed(const uint32_t* __restrict__ back, const uint32_t* __restrict__ sback,
                     const uint32_t* __restrict__ pos, const uint64_t* __restrict__ counts,
                     uint32_t G, uint64_t cap, uint64_t spill, uint64_t* __restrict__ rep) {
  __shared__ uint64_t off[FIXED_MAX_G];
  part_offsets(counts, G, off);
  const uint64_t total = (uint64_t)G * (cap + spill);
  for (uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; s < total;
       s += (uint64_t)gridDim.x * blockDim.x) {
    uint32_t p;
    uint64_t t;
    uint32_t b;
    if (s < (uint64_t)G * cap) {
      p = (uint32_t)(s / cap); t = s % cap; b = back[s];
    } else {
      const uint64_t s2 = s - (uint64_t)G * cap;
      p = (uint32_t)(s2 / spill); t = cap + s2 % spill; b = sback[s2];
    }
    if (t < counts[p]) rep[pos[off[p] + t]] = b;
  }
}

// gidx[j] = file0 + sidx[j]
extern "C" __global__ void __launch_bounds__(256)
sd_multi_gidx(const uint32_t* __restrict__ sidx, uint64_t n, uint64_t file0,
              uint64_t* __restrict__ gidx) {
  const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j < n) gidx[j] = file0 + sidx[j];
}

// out[p] = ridx[rep_pos[p]]  (rep_pos = position of the run head in the received arrays;
// group_sorted writes it indexed by received position because vals = positions)
extern "C" __global__ void __launch_bounds__(256)
sd_multi_gather(const uint32_t* __restrict__ rep_pos, const uint64_t* __restrict__ ridx,
                uint64_t m, uint64_t* __restrict__ out) {
  const uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p < m) out[p] = ridx[rep_pos[p]];
}

// rep[sidx[j]] = back[j]
extern "C" __global__ void __launch_bounds__(256)
sd_multi_scatter(const uint32_t* __restrict__ sidx, const uint64_t* __restrict__ back, uint64_t n,
                 uint64_t* __restrict__ rep) {
  const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j < n) rep[sidx[j]] = back[j];
}

hipError_t multi_splits(const uint64_t* skeys, uint64_t n, uint32_t G, uint64_t* splits,
                        hipStream_t s) {
  if (G == 0 || G > 1023) return hipErrorInvalidValue;
  sd_multi_splits<<<1, ((G + 1 + 63) / 64) * 64, 0, s>>>(skeys, n, G, splits);
  return hipGetLastError();
}

hipError_t exch_pack(const uint64_t* keys, const uint32_t* pos, uint64_t n, uint64_t file0,
                     uint32_t* rows, hipStream_t s) {
  if (n == 0) return hipSuccess;
  sd_exch_pack<<<(uint32_t)((n + 255) / 256), 256, 0, s>>>(keys, pos, n, file0, rows);
  return hipGetLastError();
}

hipError_t exch_split(const uint32_t* rows, uint64_t m, uint64_t* keys, uint32_t* vals,
                      hipStream_t s) {
  if (m == 0) return hipSuccess;
  sd_exch_split<<<(uint32_t)((m + 255) / 256), 256, 0, s>>>(rows, m, keys, vals);
  return hipGetLastError();
}

hipError_t exch_unpack(const uint32_t* back, const uint32_t* pos, uint64_t n, uint64_t* rep,
                       hipStream_t s) {
  if (n == 0) return hipSuccess;
  sd_exch_unpack<<<(uint32_t)((n + 255) / 256), 256, 0, s>>>(back, pos, n, rep);
  return hipGetLastError();
}

static uint32_t grid_for(uint64_t total) {
  const uint64_t b = (total + 255) / 256;
  return (uint32_t)(b < 65536 ? (b ? b : 1) : 65536);
}

hipError_t exch_pack_fixed(const uint64_t* keys, const uint32_t* pos, const uint64_t* counts,
                           uint32_t G, uint64_t cap, uint64_t spill, uint64_t file0, uint32_t* rows,
                           uint32_t* srows, uint32_t* overflow, hipStream_t s) {
  if (G == 0 || G > FIXED_MAX_G || cap == 0) return hipErrorInvalidValue;
  sd_exch_pack_fixed<<<grid_for((uint64_t)G * (cap + spill)), 256, 0, s>>>(
      keys, pos, counts, G, cap, spill, file0, rows, srows, overflow);
  return hipGetLastError();
}

hipError_t exch_split_fixed(const uint32_t* rows, uint64_t m, uint64_t sentinel, uint64_t* keys,
                            uint32_t* vals, uint64_t* sentinel_rows, hipStream_t s) {
  if (m == 0) return hipSuccess;
  constexpr uint64_t per = (uint64_t)SPLIT_THREADS * SPLIT_ITEMS;
  if ((m + per - 1) / per > 0xFFFFFFFFull) return hipErrorInvalidValue;
  sd_exch_split_fixed<<<(uint32_t)((m + per - 1) / per), SPLIT_THREADS, 0, s>>>(
      rows, m, sentinel, keys, vals, (unsigned long long*)sentinel_rows);
  return hipGetLastError();
}

hipError_t exch_unpack_fixed(const uint32_t* back, const uint32_t* sback, const uint32_t* pos,
                             const uint64_t* counts, uint32_t G, uint64_t cap, uint64_t spill,
                             uint64_t* rep, hipStream_t s) {
  if (G == 0 || G > FIXED_MAX_G || cap == 0) return hipErrorInvalidValue;
  sd_exch_unpack_fixed<<<grid_for((uint64_t)G * (cap + spill)), 256, 0, s>>>(
      back, sback, pos, counts, G, cap, spill, rep);
  return hipGetLastError();
}

hipError_t multi_gidx(const uint32_t* sidx, uint64_t n, uint64_t file0, uint64_t* gidx,
                      hipStream_t s) {
  if (n == 0) return hipSuccess;
  sd_multi_gidx<<<(uint32_t)((n + 255) / 256), 256, 0, s>>>(sidx, n, file0, gidx);
  return hipGetLastError();
}

hipError_t multi_gather(const uint32_t* rep_pos, const uint64_t* ridx, uint64_t m, uint64_t* out,
                        hipStream_t s) {
  if (m == 0) return hipSuccess;
  sd_multi_gather<<<(uint32_t)((m + 255) / 256), 256, 0, s>>>(rep_pos, ridx, m, out);
  return hipGetLastError();
}

hipError_t multi_scatter(const uint32_t* sidx, const uint64_t* back, uint64_t n, uint64_t* rep,
                         hipStream_t s) {
  if (n == 0) return hipSuccess;
  sd_multi_scatter<<<(uint32_t)((n + 255) / 256), 256, 0, s>>>(sidx, back, n, rep);
  return hipGetLastError();
}

}  // namespace sdcas
