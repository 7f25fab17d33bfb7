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

#include "sd_debug.h"
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

// The same for a wave of consecutive rows: one binary search for the wave's first row
// (wave-uniform: scalar loads), then each lane walks forward over the few step starts inside
// its 64-row span.  A search per lane — 17 dependent loads at 100 K steps — was most of the
// decision kernel's time at 10 M rows.
__device__ __forceinline__ uint32_t wave_step_of(const uint32_t* starts, uint32_t nsteps,
                                                 uint32_t i0, uint32_t i) {
  uint32_t k = step_of(starts, nsteps, __builtin_amdgcn_readfirstlane(i0));
  while (starts[k + 1] <= i) ++k;  // starts[nsteps] = sentinel
  return k;
}

// Rows that already own an Object (sd_links_pre_*, below): the event list sorted by (key,
// row) — ekeys / erows — and T[j] = the smallest pre-existing Object over the key's events in
// steps up to event j's; a row's own value is T at its key's last event with row < bound
// (the first row of the next step), found by one binary search over (key, row) order.
struct PreEvents {
  const uint64_t* ekeys;
  const uint32_t* erows;
  const uint64_t* T;       // scan elements: low 32 bits
  const uint32_t* filter;  // bitmap of mix(key) over the events' keys (FILTER_BITS bits)
  uint64_t m;
};
constexpr uint32_t FILTER_BITS = 23;  // 1 MiB: ~1 % false positives at 100 K events
__device__ __forceinline__ uint32_t filter_bit(uint64_t key) {
  uint64_t z = key * 0x9E3779B97F4A7C15ull;
  return (uint32_t)(z >> (64 - FILTER_BITS));
}
__device__ __forceinline__ uint32_t pre_min_of(const PreEvents& ev, uint64_t key, uint32_t bound) {
  const uint32_t bit = filter_bit(key);
  if (!((ev.filter[bit >> 5] >> (bit & 31u)) & 1u)) return 0xFFFFFFFFu;
  uint64_t lo = 0, hi = ev.m;  // first element not < (key, bound)
  while (lo < hi) {
    const uint64_t mid = (lo + hi) >> 1;
    const uint64_t k = ev.ekeys[mid];
    if (k < key || (k == key && ev.erows[mid] < bound)) lo = mid + 1; else hi = mid;
  }
  return lo > 0 && ev.ekeys[lo - 1] == key ? (uint32_t)ev.T[lo - 1] : 0xFFFFFFFFu;
}

// Per-row decision (mod.rs:202-347 replayed with HashMap order := ascending row):
//   hashed, key held by an Object that existed before the job (seeded: rep < ROW_FLAG is the
//           lowest such Object id; ev: the lowest pre-existing Object of a row with the key in
//           this step or an earlier one, sd_links_pre_*): EXISTING — the step's find_many
//           returns it (:180-198, no location filter), find() picks the first Object in id
//           order (:214-224) and the key never creates (:246-253);
//   hashed: CREATED iff its key's first row (rep) is in the same step — no intra-step dedup,
//           mod.rs:246-311 — else LINKED to the Object of rep (find() = the lowest Object
//           id, created for the key's lowest row, :214-224).  The first row r <= i is a hashed
//           row, never a re-queried one, so it shares i's step iff r >= starts[step];
//   no cas_id (empty): CREATED, its own Object (:248-253);
//   error: DROPPED (:125-141);  rows past the last step: NOT_REACHED.
// counts[2k] / counts[2k+1] += created / linked rows whose final step is k.
extern "C" __global__ void __launch_bounds__(256)
sd_links_decide(const uint8_t* __restrict__ state, const uint32_t* __restrict__ rep, uint64_t n,
                const uint32_t* __restrict__ starts, uint32_t nsteps, uint64_t reached,
                uint32_t* __restrict__ step_out, uint32_t* __restrict__ object_out,
                uint8_t* __restrict__ action_out, unsigned int* __restrict__ counts, bool seeded,
                const uint64_t* __restrict__ keys, PreEvents ev, uint32_t chunk) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t i0 = i - (threadIdx.x & 63u);  // the wave's first row
  uint32_t step = SD_LINKS_NO_STEP, object = SD_LINKS_NO_OBJECT;
  uint8_t action = SD_LINKS_NOT_REACHED;
  if (i0 < n && i0 < reached) {  // (uniform) rows of a wave straddling `reached` search too
    const uint32_t k = wave_step_of(starts, nsteps, (uint32_t)i0,
                                    (uint32_t)(i < reached ? i : reached - 1));
    if (i < n && i < reached) step = k;
  }
  if (step != SD_LINKS_NO_STEP) {
    const uint8_t st = state ? state[i] : (uint8_t)SD_LINKS_HASHED;
    if (st == SD_LINKS_ERROR) {
      action = SD_LINKS_DROPPED;
    } else if (st == SD_LINKS_NO_CAS) {
      action = SD_LINKS_CREATED;
      object = (uint32_t)i;
    } else {
      uint32_t v = rep[i];
      const uint32_t r = seeded ? v & ~LINKS_ROW_FLAG : v;  // the key's first row
      // INVARIANT (both uses below: pre_min_of's bound = starts[step + 1], and the CREATED
      // test r >= starts[step]): a HASHED row is never a re-queried cursor row — only a row
      // that stays orphan (an error, or an empty file with no cas_id) is the last row of one
      // step and the first of the next (starts[k] == starts[k-1] + chunk - 1).  If "stays
      // orphan" ever grows to include hashed rows, both tests misclassify such rows; the
      // debug build checks it for this row.
      SD_DBG_CHECK(!(step > 0 && (uint32_t)i == starts[step] && starts[step] + 1u == starts[step - 1] + chunk),
                   "links: hashed row %u is the re-queried first row of step %u", (uint32_t)i, step);
      if (ev.m) {  // a pre-existing Object its step or an earlier one saw
        const uint32_t bound = step + 1 < nsteps ? starts[step + 1] : 0xFFFFFFFFu;
        v = min(v, pre_min_of(ev, keys[i], bound));
      }
      if (seeded && v < LINKS_ROW_FLAG) {
        action = SD_LINKS_EXISTING;
        object = v;
      } else if (r == (uint32_t)i || r >= starts[step]) {
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

// ---- rows that already own an Object (object_id set, cas_id NULL) -----------------------
// The orphan query takes `object_id IS NULL OR cas_id IS NULL` (file_identifier_job.rs:
// 258-261), so a file_path the watcher gave an Object while it was still empty and that was
// written afterwards (watcher/utils.rs:236-293 creates the Object; :473-490 writes the old,
// NULL cas_id back with the new size) is a row whose Object P exists before the job.  Its
// step writes its cas_id X first (mod.rs:157-178), so that step's find_many (:180-198) sees P
// under X: every row of the step with X links to the smallest Object id carrying X and X
// never creates (:214-224, :246-253).  A later step still sees P when it won (its row stays
// connected to it); when a smaller Object won, P lost the row — but then the smaller one
// stays, so what each row needs is the smallest P over the key's rows in its own or an
// earlier step.  Only those rows' events matter, and they are few (a create-then-write is
// the exception, not the rule), so the work is on the EVENT list (hashed, reached rows with
// an Object), not on every row:
//   1. ordered compaction of the events: (key, row), row order kept (count / scan / emit);
//   2. a stable sort of the events by key (sd_cas_sort_pairs_dev): (key, row) order;
//   3. forward segmented min over the events, segments = keys:   F[j] = min P up to j;
//      backward, segments = (key, step) run ends:  T[j] = F[end of j's run]
//      (scan element: bit 63 = segment start, low 32 bits = value, 0xFFFFFFFF = none);
//   4. each hashed row looks its key up (a 1 MiB bitmap of the events' keys first, then one
//      binary search over (key, row) order) in the decision kernel above.
constexpr uint64_t SEG_START = 1ull << 63;
constexpr uint64_t SEG_NONE = 0xFFFFFFFFull;  // the identity: no start, no Object
__device__ __forceinline__ uint64_t segmin(uint64_t a, uint64_t b) {
  if (b & SEG_START) return b;
  const uint32_t va = (uint32_t)a, vb = (uint32_t)b;
  return (a & SEG_START) | (uint64_t)(va < vb ? va : vb);
}
__device__ __forceinline__ uint64_t shfl_up64(uint64_t x, int d) {
  const uint32_t lo = __shfl_up((uint32_t)x, d, 64), hi = __shfl_up((uint32_t)(x >> 32), d, 64);
  return ((uint64_t)hi << 32) | lo;
}

// Any seeded or pre-existing Object id >= 2^31 (the row tag of the seeded grouping) sets
// *bad; SD_LINKS_NO_OBJECT is allowed where `none_ok` (a row without an Object).
extern "C" __global__ void __launch_bounds__(256)
sd_links_check_ids(const uint32_t* __restrict__ ids, uint64_t n, uint32_t none_ok,
                   unsigned long long* __restrict__ bad) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  bool b = false;
  if (i < n) {
    const uint32_t v = ids[i];
    b = v >= LINKS_ROW_FLAG && !(none_ok && v == SD_LINKS_NO_OBJECT);
  }
  if (__ballot(b) && (threadIdx.x & 63u) == 0) atomicAdd(bad, 1ull);
}

// 1. ordered compaction of the events.  A workgroup takes EV_ROWS rows; count: its events
// (ballots); the block counts' exclusive scan (one workgroup); emit: the events in row order
// at the block's offset, and each event key's bit in the filter.
constexpr int EV_THREADS = 1024, EV_ITEMS = 16;
constexpr uint64_t EV_ROWS = (uint64_t)EV_THREADS * EV_ITEMS;
__device__ __forceinline__ bool is_event(const uint8_t* state, const uint32_t* pre, uint64_t i,
                                         uint64_t reached) {
  return i < reached && (!state || state[i] == SD_LINKS_HASHED) && pre[i] != SD_LINKS_NO_OBJECT;
}

extern "C" __global__ void __launch_bounds__(EV_THREADS)
sd_links_pre_count(const uint8_t* __restrict__ state, const uint32_t* __restrict__ pre,
                   uint64_t reached, uint32_t* __restrict__ bcount) {
  __shared__ uint32_t wsum[EV_THREADS / 64];
  uint32_t c = 0;
  for (int u = 0; u < EV_ITEMS; ++u) {
    const uint64_t i = blockIdx.x * EV_ROWS + (uint64_t)u * EV_THREADS + threadIdx.x;
    c += (uint32_t)__popcll(__ballot(is_event(state, pre, i, reached)));
  }
  if ((threadIdx.x & 63u) == 0) wsum[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t t = 0;
    for (int w = 0; w < EV_THREADS / 64; ++w) t += wsum[w];
    bcount[blockIdx.x] = t;
  }
}

// one workgroup: bcount[b] := sum of bcount[0..b) in place, total -> *total
extern "C" __global__ void __launch_bounds__(256)
sd_links_pre_bscan(uint32_t* __restrict__ bcount, uint64_t nb, unsigned long long* __restrict__ total) {
  __shared__ uint32_t wsum[4];
  uint64_t carry = 0;
  const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
  for (uint64_t base = 0; base < nb; base += 256) {
    const uint64_t b = base + threadIdx.x;
    const uint32_t x = b < nb ? bcount[b] : 0u;
    uint32_t inc = x;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint32_t y = __shfl_up(inc, d, 64);
      if (lane >= (uint32_t)d) inc += y;
    }
    if (lane == 63) wsum[w] = inc;
    __syncthreads();
    uint32_t before = 0, all = 0;
    for (uint32_t k = 0; k < 4; ++k) {
      if (k < w) before += wsum[k];
      all += wsum[k];
    }
    if (b < nb) bcount[b] = (uint32_t)(carry + before + inc - x);
    carry += all;
    __syncthreads();  // wsum is rewritten by the next round
  }
  if (threadIdx.x == 0) *total = carry;
}

extern "C" __global__ void __launch_bounds__(EV_THREADS)
sd_links_pre_emit(const uint64_t* __restrict__ keys, const uint8_t* __restrict__ state,
                  const uint32_t* __restrict__ pre, uint64_t reached,
                  const uint32_t* __restrict__ boff, uint64_t* __restrict__ ekeys,
                  uint32_t* __restrict__ erows, uint32_t* __restrict__ filter) {
  __shared__ uint32_t wbase[EV_ITEMS][EV_THREADS / 64];
  const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
  const uint64_t below = (1ull << lane) - 1ull;
  uint64_t m[EV_ITEMS];
  for (int u = 0; u < EV_ITEMS; ++u) {
    const uint64_t i = blockIdx.x * EV_ROWS + (uint64_t)u * EV_THREADS + threadIdx.x;
    m[u] = __ballot(is_event(state, pre, i, reached));
    if (lane == 0) wbase[u][w] = (uint32_t)__popcll(m[u]);
  }
  __syncthreads();
  if (threadIdx.x == 0) {  // row order = (u, wave) order: exclusive prefix in place
    uint32_t t = boff[blockIdx.x];
    for (int u = 0; u < EV_ITEMS; ++u)
      for (int k = 0; k < EV_THREADS / 64; ++k) {
        const uint32_t c = wbase[u][k];
        wbase[u][k] = t;
        t += c;
      }
  }
  __syncthreads();
  for (int u = 0; u < EV_ITEMS; ++u) {
    if (!((m[u] >> lane) & 1ull)) continue;
    const uint64_t i = blockIdx.x * EV_ROWS + (uint64_t)u * EV_THREADS + threadIdx.x;
    const uint32_t d = wbase[u][w] + (uint32_t)__popcll(m[u] & below);
    const uint64_t k = keys[i];
    ekeys[d] = k;
    erows[d] = (uint32_t)i;
    const uint32_t bit = filter_bit(k);
    atomicOr(&filter[bit >> 5], 1u << (bit & 31u));
  }
}

// 3. over the m sorted events (skeys, srows): value = the row's Object, start = first event
// of its key
extern "C" __global__ void __launch_bounds__(256)
sd_links_pre_mark(const uint64_t* __restrict__ skeys, const uint32_t* __restrict__ srows,
                  const uint32_t* __restrict__ pre, uint64_t m, uint64_t* __restrict__ elem) {
  const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= m) return;
  elem[j] = (j == 0 || skeys[j] != skeys[j - 1] ? SEG_START : 0ull) | (uint64_t)pre[srows[j]];
}

// F -> the backward scan's input, in place: a (key, step) run's last element carries F as a
// segment start, every other element the identity
extern "C" __global__ void __launch_bounds__(256)
sd_links_pre_runs(const uint64_t* __restrict__ skeys, const uint32_t* __restrict__ srows,
                  const uint32_t* __restrict__ starts, uint32_t nsteps, uint64_t m,
                  uint64_t* __restrict__ elem) {
  const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= m) return;
  bool end = j + 1 == m || skeys[j] != skeys[j + 1];
  if (!end) {  // the next event of the key is in a later step iff it is past this step's end
    const uint32_t k = step_of(starts, nsteps, srows[j]);
    end = k + 1 < nsteps && srows[j + 1] >= starts[k + 1];
  }
  elem[j] = end ? (SEG_START | (elem[j] & SEG_NONE)) : SEG_NONE;
}

// Device-wide inclusive segmented-min scan in three launches (reduce-then-scan): each
// workgroup scans a tile of SCAN_TILE elements and leaves the tile's total; one workgroup
// scans the totals (exclusive); every tile but the first folds its prefix in.  `reverse`
// scans from the last element to the first (logical k = physical n-1-k).
constexpr int SCAN_THREADS = 256, SCAN_ITEMS = 8;
constexpr uint64_t SCAN_TILE = (uint64_t)SCAN_THREADS * SCAN_ITEMS;

// workgroup scan of one value per thread: returns the thread's EXCLUSIVE prefix and (in
// *total) the workgroup's total; the closing barrier lets the caller reuse wsum
__device__ __forceinline__ uint64_t block_segmin_excl(uint64_t x, uint64_t* wsum, uint64_t* total) {
  const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
  uint64_t inc = x;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint64_t y = shfl_up64(inc, d);
    if (lane >= (uint32_t)d) inc = segmin(y, inc);
  }
  if (lane == 63) wsum[w] = inc;
  __syncthreads();
  uint64_t excl = SEG_NONE, all = SEG_NONE;
  for (uint32_t k = 0; k < SCAN_THREADS / 64; ++k) {
    if (k == w) excl = all;
    all = segmin(all, wsum[k]);
  }
  const uint64_t prev = shfl_up64(inc, 1);
  if (lane) excl = segmin(excl, prev);
  *total = all;
  __syncthreads();
  return excl;
}

extern "C" __global__ void __launch_bounds__(SCAN_THREADS)
sd_segmin_tiles(uint64_t* __restrict__ data, uint64_t n, int reverse, uint64_t* __restrict__ tiles) {
  __shared__ uint64_t wsum[SCAN_THREADS / 64];
  const uint64_t k0 = (uint64_t)blockIdx.x * SCAN_TILE + (uint64_t)threadIdx.x * SCAN_ITEMS;
  uint64_t v[SCAN_ITEMS], acc = SEG_NONE;
#pragma unroll
  for (int u = 0; u < SCAN_ITEMS; ++u) {
    const uint64_t k = k0 + u;
    v[u] = k < n ? data[reverse ? n - 1 - k : k] : SEG_NONE;
    acc = segmin(acc, v[u]);
  }
  uint64_t total;
  uint64_t run = block_segmin_excl(acc, wsum, &total);
#pragma unroll
  for (int u = 0; u < SCAN_ITEMS; ++u) {
    const uint64_t k = k0 + u;
    run = segmin(run, v[u]);
    if (k < n) data[reverse ? n - 1 - k : k] = run;
  }
  if (threadIdx.x == 0) tiles[blockIdx.x] = total;
}

// one workgroup: tiles[t] := the fold of tiles[0..t) (exclusive), in place
extern "C" __global__ void __launch_bounds__(SCAN_THREADS)
sd_segmin_tile_prefix(uint64_t* __restrict__ tiles, uint64_t ntiles) {
  __shared__ uint64_t wsum[SCAN_THREADS / 64];
  uint64_t carry = SEG_NONE;
  for (uint64_t b = 0; b < ntiles; b += SCAN_THREADS) {
    const uint64_t t = b + threadIdx.x;
    const uint64_t x = t < ntiles ? tiles[t] : SEG_NONE;
    uint64_t total;
    const uint64_t excl = block_segmin_excl(x, wsum, &total);
    if (t < ntiles) tiles[t] = segmin(carry, excl);
    carry = segmin(carry, total);
  }
}

extern "C" __global__ void __launch_bounds__(SCAN_THREADS)
sd_segmin_fix(uint64_t* __restrict__ data, uint64_t n, int reverse, const uint64_t* __restrict__ tiles) {
  const uint64_t t = blockIdx.x + 1;  // tile 0 has nothing before it
  const uint64_t pre = tiles[t];
  for (uint64_t u = threadIdx.x; u < SCAN_TILE; u += SCAN_THREADS) {
    const uint64_t k = t * SCAN_TILE + u;
    if (k >= n) break;
    const uint64_t p = reverse ? n - 1 - k : k;
    data[p] = segmin(pre, data[p]);
  }
}

hipError_t segmin_scan(uint64_t* data, uint64_t n, bool reverse, uint64_t* tiles, hipStream_t s) {
  if (n == 0) return hipSuccess;
  const uint64_t nt = (n + SCAN_TILE - 1) / SCAN_TILE;
  sd_segmin_tiles<<<(uint32_t)nt, SCAN_THREADS, 0, s>>>(data, n, reverse ? 1 : 0, tiles);
  if (nt > 1) {
    sd_segmin_tile_prefix<<<1, SCAN_THREADS, 0, s>>>(tiles, nt);
    sd_segmin_fix<<<(uint32_t)(nt - 1), SCAN_THREADS, 0, s>>>(data, n, reverse ? 1 : 0, tiles);
  }
  return hipGetLastError();
}

size_t segmin_tiles_bytes(uint64_t n) { return ((n + SCAN_TILE - 1) / SCAN_TILE + 1) * 8; }
size_t pre_blocks(uint64_t n) { return (n + EV_ROWS - 1) / EV_ROWS; }
size_t pre_filter_bytes() { return ((size_t)1 << FILTER_BITS) / 8; }

hipError_t links_check_ids(const uint32_t* ids, uint64_t n, bool none_ok, uint64_t* d_bad,
                           hipStream_t s) {
  if (n == 0) return hipSuccess;
  sd_links_check_ids<<<(uint32_t)((n + 255) / 256), 256, 0, s>>>(ids, n, none_ok ? 1u : 0u,
                                                                (unsigned long long*)d_bad);
  return hipGetLastError();
}

hipError_t links_pre_count(const uint8_t* state, const uint32_t* pre, uint64_t reached,
                           uint32_t* bcount, uint64_t* d_total, hipStream_t s) {
  const uint64_t nb = pre_blocks(reached);
  if (nb == 0) return hipMemsetAsync(d_total, 0, 8, s);
  sd_links_pre_count<<<(uint32_t)nb, EV_THREADS, 0, s>>>(state, pre, reached, bcount);
  sd_links_pre_bscan<<<1, 256, 0, s>>>(bcount, nb, (unsigned long long*)d_total);
  return hipGetLastError();
}

hipError_t links_pre_emit(const uint64_t* keys, const uint8_t* state, const uint32_t* pre,
                          uint64_t reached, const uint32_t* boff, uint64_t* ekeys,
                          uint32_t* erows, uint32_t* filter, hipStream_t s) {
  const uint64_t nb = pre_blocks(reached);
  if (nb == 0) return hipSuccess;
  sd_links_pre_emit<<<(uint32_t)nb, EV_THREADS, 0, s>>>(keys, state, pre, reached, boff, ekeys,
                                                        erows, filter);
  return hipGetLastError();
}

hipError_t links_pre_scan(const uint64_t* skeys, const uint32_t* srows, const uint32_t* pre,
                          uint64_t m, const uint32_t* starts, uint32_t nsteps, uint64_t* elem,
                          uint64_t* tiles, hipStream_t s) {
  if (m == 0) return hipSuccess;
  const uint32_t g = (uint32_t)((m + 255) / 256);
  sd_links_pre_mark<<<g, 256, 0, s>>>(skeys, srows, pre, m, elem);
  hipError_t e = segmin_scan(elem, m, false, tiles, s);
  if (e != hipSuccess) return e;
  sd_links_pre_runs<<<g, 256, 0, s>>>(skeys, srows, starts, nsteps, m, elem);
  return segmin_scan(elem, m, true, tiles, s);
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
                        uint32_t* counts, bool seeded, const uint64_t* keys,
                        const uint64_t* ekeys, const uint32_t* erows, const uint64_t* T,
                        const uint32_t* filter, uint64_t m, uint32_t chunk, hipStream_t s) {
  if (n == 0) return hipSuccess;
  PreEvents ev{ekeys, erows, T, filter, m};
  sd_links_decide<<<(uint32_t)((n + 255) / 256), 256, 0, s>>>(
      state, rep, n, starts, nsteps, reached, step_out, object_out, action_out, counts, seeded,
      keys, ev, chunk);
  return hipGetLastError();
}

SD_DBG_ACCESSOR(sd_dbg_violations_links)

}  // namespace sdcas
