// links.hip — Object-link emission of the file identifier job on gfx950.
//
// The reference decides, per job step of CHUNK_SIZE orphan rows (file_identifier_job.rs:
// 180-236, identifier_job_step mod.rs:98-350): which rows get their cas_id written
// (:157-178), which link to an existing Object (:202-238), which get a new Object via
// create_many (:246-347), and the step's (total_created, total_linked) (:349).  Given the
// step of every row (host: the cursor walk, see sd_cas_identifier_links_dev) and the
// canonical representative of every hashed row (the grouping), each decision is a per-row
// function — one elementwise pass here, with the per-step counts reduced by wave ballots.
// Integer work bound by HBM (a few bytes per row); nothing is reshaped into a GEMM.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "sd_links.h"

namespace sdcas {

// Split the rows by state: hashed rows -> (key, row) pairs for the grouping; every other
// row -> (row << 8 | state) for the host's cursor walk (they stay orphan after a step).
// Both lists are unordered (the grouping's minimum does not depend on the order; the host
// sorts the orphans).  A workgroup takes SPLIT_ROWS rows, counts them per wave with ballots,
// and reserves its runs with ONE device atomic per list: appending per wave (one returning
// atomic per 64 rows on one counter) took 2 ms of a 10 M-row job — same-address device
// atomics complete one per ~12.8 ns (tools/ubench_bucketload.hip).
constexpr int SPLIT_THREADS = 1024, SPLIT_ITEMS = 16;
constexpr uint32_t SPLIT_ROWS = SPLIT_THREADS * SPLIT_ITEMS;
constexpr int SPLIT_WAVES = SPLIT_THREADS / 64;
extern "C" __global__ void __launch_bounds__(SPLIT_THREADS)
sd_links_split(const uint64_t* __restrict__ keys, const uint8_t* __restrict__ state, uint64_t n,
               uint64_t* __restrict__ hkeys, uint32_t* __restrict__ hrows,
               unsigned long long* __restrict__ hcount, uint64_t* __restrict__ orphans,
               unsigned long long* __restrict__ ocount, uint32_t row_flag) {
  __shared__ uint32_t wh[SPLIT_WAVES], wo[SPLIT_WAVES];
  __shared__ unsigned long long base[2];
  const uint64_t row0 = (uint64_t)blockIdx.x * SPLIT_ROWS;
  const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
  const uint64_t below = (1ull << lane) - 1ull;
  uint8_t st[SPLIT_ITEMS];
  uint32_t th = 0, to = 0;  // the wave's hashed / orphan rows
#pragma unroll
  for (int j = 0; j < SPLIT_ITEMS; ++j) {
    const uint64_t i = row0 + (uint64_t)j * SPLIT_THREADS + threadIdx.x;
    st[j] = i < n && state ? state[i] : (uint8_t)SD_LINKS_HASHED;
  }
#pragma unroll
  for (int j = 0; j < SPLIT_ITEMS; ++j) {
    const bool valid = row0 + (uint64_t)j * SPLIT_THREADS + threadIdx.x < n;
    th += (uint32_t)__popcll(__ballot(valid && st[j] == SD_LINKS_HASHED));
    to += (uint32_t)__popcll(__ballot(valid && st[j] != SD_LINKS_HASHED));
  }
  if (lane == 0) { wh[w] = th; wo[w] = to; }
  __syncthreads();
  if (threadIdx.x == 0) {  // wave prefixes in place, then the block's two runs
    uint32_t ph = 0, po = 0;
    for (int k = 0; k < SPLIT_WAVES; ++k) {
      const uint32_t a = wh[k], b = wo[k];
      wh[k] = ph; wo[k] = po;
      ph += a; po += b;
    }
    base[0] = ph ? atomicAdd(hcount, (unsigned long long)ph) : 0ull;
    base[1] = po ? atomicAdd(ocount, (unsigned long long)po) : 0ull;
  }
  __syncthreads();
  uint64_t h = base[0] + wh[w], o = base[1] + wo[w];
#pragma unroll
  for (int j = 0; j < SPLIT_ITEMS; ++j) {
    const uint64_t i = row0 + (uint64_t)j * SPLIT_THREADS + threadIdx.x;
    const bool valid = i < n;
    const bool hashed = valid && st[j] == SD_LINKS_HASHED, orphan = valid && st[j] != SD_LINKS_HASHED;
    const uint64_t hm = __ballot(hashed), om = __ballot(orphan);
    if (hashed) {
      const uint64_t d = h + (uint64_t)__popcll(hm & below);
      hkeys[d] = keys[i];
      hrows[d] = (uint32_t)i | row_flag;
    }
    if (orphan) orphans[o + (uint64_t)__popcll(om & below)] = (i << 8) | st[j];
    h += (uint64_t)__popcll(hm);
    o += (uint64_t)__popcll(om);
  }
}

extern "C" __global__ void __launch_bounds__(256)
sd_links_scatter(const uint32_t* __restrict__ minrow, const uint32_t* __restrict__ hrows,
                 uint64_t m, uint32_t* __restrict__ rep, uint32_t row_flag) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < m) rep[hrows[i] & ~row_flag] = minrow[i];
}

// Final step of row i = the largest k with starts[k] <= i (steps are consecutive windows
// [starts[k], starts[k] + chunk) that overlap by at most the re-queried cursor row).
__device__ __forceinline__ uint32_t step_of(const uint32_t* starts, uint32_t nsteps, uint32_t i) {
  uint32_t lo = 0, hi = nsteps;  // starts[lo] <= i < starts[hi] (starts[nsteps] = sentinel)
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (starts[mid] <= i) lo = mid; else hi = mid;
  }
  return lo;
}

// Per-row decision (mod.rs:202-347 replayed with HashMap order := ascending row):
//   hashed, key held by an Object that existed before the job (seeded: rep < ROW_FLAG is the
//           lowest such Object id): EXISTING — the step's find_many returns it (:180-198, no
//           location filter), find() picks the first Object in id order (:214-224) and the
//           key never creates (:246-253);
//   hashed: CREATED iff its key's first row (rep) is in the same step — no intra-step dedup,
//           mod.rs:246-311 — else LINKED to the Object of rep (find() = the lowest Object
//           id, created for the key's lowest row, :214-224);
//   no cas_id (empty): CREATED, its own Object (:248-253);
//   error: DROPPED (:125-141);  rows past the last step: NOT_REACHED.
// counts[2k] / counts[2k+1] += created / linked rows whose final step is k.
extern "C" __global__ void __launch_bounds__(256)
sd_links_decide(const uint8_t* __restrict__ state, const uint32_t* __restrict__ rep, uint64_t n,
                const uint32_t* __restrict__ starts, uint32_t nsteps, uint64_t reached,
                uint32_t* __restrict__ step_out, uint32_t* __restrict__ object_out,
                uint8_t* __restrict__ action_out, unsigned int* __restrict__ counts, bool seeded) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t step = SD_LINKS_NO_STEP, object = SD_LINKS_NO_OBJECT;
  uint8_t action = SD_LINKS_NOT_REACHED;
  if (i < n && i < reached) {
    const uint8_t st = state ? state[i] : (uint8_t)SD_LINKS_HASHED;
    step = step_of(starts, nsteps, (uint32_t)i);
    if (st == SD_LINKS_ERROR) {
      action = SD_LINKS_DROPPED;
    } else if (st == SD_LINKS_NO_CAS) {
      action = SD_LINKS_CREATED;
      object = (uint32_t)i;
    } else {
      const uint32_t v = rep[i];
      const uint32_t r = seeded ? v & ~LINKS_ROW_FLAG : v;  // the key's first row
      if (seeded && v < LINKS_ROW_FLAG) {
        action = SD_LINKS_EXISTING;
        object = v;
      } else if (r == (uint32_t)i || step_of(starts, nsteps, r) == step) {
        action = SD_LINKS_CREATED;
        object = (uint32_t)i;
      } else {
        action = SD_LINKS_LINKED;
        object = r;
      }
    }
  }
  if (i < n) {
    step_out[i] = step;
    object_out[i] = object;
    action_out[i] = action;
  }
  // per-step counts: runs of equal steps inside a wave are the common case (steps are
  // CHUNK_SIZE rows wide), so count per (wave, step) with ballots and one atomic per run
  const bool created = action == SD_LINKS_CREATED,
             linked = action == SD_LINKS_LINKED || action == SD_LINKS_EXISTING;
  uint64_t todo = __ballot(created || linked);
  const uint32_t lane = threadIdx.x & 63u;
  while (todo) {
    const uint32_t leader = (uint32_t)__ffsll((unsigned long long)todo) - 1u;
    const uint32_t s = __shfl(step, (int)leader, 64);
    const uint64_t same = __ballot((created || linked) && step == s);
    const uint64_t c = __ballot(created && step == s), l = __ballot(linked && step == s);
    if (lane == leader) {
      if (c) atomicAdd(&counts[2 * (uint64_t)s], (unsigned int)__popcll(c));
      if (l) atomicAdd(&counts[2 * (uint64_t)s + 1], (unsigned int)__popcll(l));
    }
    todo &= ~same;
  }
}

hipError_t links_split(const uint64_t* keys, const uint8_t* state, uint64_t n, uint64_t* hkeys,
                       uint32_t* hrows, uint64_t* d_hcount, uint64_t* orphans, uint64_t* d_ocount,
                       uint32_t row_flag, hipStream_t s) {
  if (n == 0) return hipSuccess;
  sd_links_split<<<(uint32_t)((n + SPLIT_ROWS - 1) / SPLIT_ROWS), SPLIT_THREADS, 0, s>>>(
      keys, state, n, hkeys, hrows, (unsigned long long*)d_hcount, orphans,
      (unsigned long long*)d_ocount, row_flag);
  return hipGetLastError();
}

hipError_t links_scatter(const uint32_t* minrow, const uint32_t* hrows, uint64_t m, uint32_t* rep,
                         uint32_t row_flag, hipStream_t s) {
  if (m == 0) return hipSuccess;
  sd_links_scatter<<<(uint32_t)((m + 255) / 256), 256, 0, s>>>(minrow, hrows, m, rep, row_flag);
  return hipGetLastError();
}

hipError_t links_decide(const uint8_t* state, const uint32_t* rep, uint64_t n,
                        const uint32_t* starts, uint32_t nsteps, uint64_t reached,
                        uint32_t* step_out, uint32_t* object_out, uint8_t* action_out,
                        uint32_t* counts, bool seeded, hipStream_t s) {
  if (n == 0) return hipSuccess;
  sd_links_decide<<<(uint32_t)((n + 255) / 256), 256, 0, s>>>(
      state, rep, n, starts, nsteps, reached, step_out, object_out, action_out, counts, seeded);
  return hipGetLastError();
}

}  // namespace sdcas
