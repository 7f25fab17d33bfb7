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
