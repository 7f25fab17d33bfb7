// sd_group.h — host-side launchers for the sort / grouping kernels (group.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace sdcas {

// Workspace bytes needed by radix_sort_pairs / group_keys for n keys.
size_t sort_workspace_bytes(uint64_t n);
size_t group_workspace_bytes(uint64_t n);

// Stable LSD sort of (keys, vals) on bits [begin_bit, end_bit).  vals_in == nullptr means
// vals = 0..n-1.  Results land in (keys_out, vals_out).  keys_in is not modified;
// `ws` must hold sort_workspace_bytes(n).  n < 2^32.  iota_out (vals_in == nullptr only):
// iota_out[i] = i is written by the first pass as well (group_sorted's rep_prefilled).
hipError_t radix_sort_pairs(const uint64_t* keys_in, const uint32_t* vals_in, uint64_t* keys_out,
                            uint32_t* vals_out, uint64_t n, int begin_bit, int end_bit,
                            void* ws, hipStream_t stream, uint32_t* iota_out = nullptr);

// Canonical grouping: rep[i] = min{ j : keys[j] == keys[i] }; *d_objects = #distinct keys
// (written on the device).  ws must hold group_workspace_bytes(n).
hipError_t group_keys(const uint64_t* keys, uint64_t n, uint32_t* rep, uint64_t* d_objects,
                      void* ws, hipStream_t stream);

// out[i] = min{ val(j) : keys[j] == keys[i] } by two stable LSD sorts (the fallback of
// hash_group_min beyond its range); ws: group_min_sorted_workspace_bytes(n).
size_t group_min_sorted_workspace_bytes(uint64_t n);
hipError_t group_min_by_sort(const uint64_t* keys, const uint32_t* vals, uint64_t n, uint32_t* out,
                             uint64_t* d_objects, void* ws, hipStream_t stream);

// Group already-sorted pairs (keys ascending, vals = original idx, stable): rep[v] = the val
// of v's run head.  rep_prefilled: rep[v] == v already holds for every val (vals a
// permutation of 0..n-1 and rep laid down by the iota sort), so heads are not stored.
hipError_t group_sorted(const uint64_t* skeys, const uint32_t* svals, uint64_t n, uint32_t* rep,
                        uint64_t* d_objects, void* ws, hipStream_t stream, bool rep_prefilled = false);

// Device-wide exclusive scan of m <= 4096^2 u32 (partial: >= m/4096 + 1 u32 of scratch).
// total (optional, device): the sum of in[] in u64 — exact even where the u32 scan wraps.
hipError_t exclusive_scan_u32(const uint32_t* in, uint32_t* out, uint64_t m, uint32_t* partial,
                              hipStream_t stream, unsigned long long* total = nullptr);

// ---- group_hash.hip: grouping without a full sort -------------------------------------
bool hash_group_supported(uint64_t n);
// target = mean keys per final bucket (0 = the tuned default, 1,536); smaller targets give
// deeper partitions (tests use them to reach the > 200M-key plan shapes at small n)
size_t hash_group_workspace_bytes(uint64_t n, uint64_t target = 0);
size_t partition_workspace_bytes(uint64_t n, uint32_t parts);
// out[i] = min{ val(j) : keys[j] == keys[i] } with val(j) = vals ? vals[j] : j;
// *d_objects = #distinct keys (written on the device).  n < 2^32.  `totals`: a persistent
// device buffer of GROUP_TOTALS_WORDS u32, all zero before the first call (every call leaves
// it zero again); calls using it must be stream-ordered.
constexpr uint32_t GROUP_TOTALS_WORDS = 33 * 1024;
hipError_t hash_group_min(const uint64_t* keys, const uint32_t* vals, uint64_t n, uint32_t* out,
                          uint64_t* d_objects, void* ws, uint32_t* totals, hipStream_t stream,
                          uint64_t target = 0);
// The fused hash + group chain (K1G writes the regions, sd_bucket_min_regions groups them):
// n <= 1,441,792 keys; regions of region_capacity(n) rows per coarse bucket; `cursor`
// (REGIONS u32, persistent, zero between calls) is re-zeroed by the bucket tables.
uint64_t region_capacity(uint64_t n);
bool region_group_supported(uint64_t n);
size_t region_group_workspace_bytes(uint64_t n);
void region_group_layout(void* ws, uint64_t n, uint64_t** rkeys, uint32_t** rfile, uint64_t** gkeys,
                         uint32_t** gvals, uint64_t** spill_keys, uint32_t** spill_file);
// cursor: the set's REGION_SET_WORDS counters (sd_mix.h); d_objects: 2 u64 (count, overflow
// carve cursor; K1G zeroed both); spill_keys/spill_file: the rows K1G could not store in
// their region; keys/n: the batch's key array, read only if a full region's distinct keys
// overflow its LDS table; fill_limit: 0, or (tests) a lower distinct-key bound for the LDS
// tables so their overflow paths run
hipError_t region_group_min(const uint64_t* rkeys, const uint32_t* rfile, uint32_t* cursor,
                            uint64_t cap, uint32_t* out, uint64_t* d_objects, uint64_t* gkeys,
                            uint32_t* gvals, const uint64_t* keys, uint64_t n,
                            const uint64_t* spill_keys, const uint32_t* spill_file,
                            uint32_t fill_limit, hipStream_t stream);
// Key-range partition: part(k) = floor(k * parts / 2^64); out_keys/out_pos hold the keys and
// their input positions part-contiguous (order inside a part unspecified), d_counts[p] the
// part sizes.  ws: partition_workspace_bytes(n, parts).
hipError_t partition_range(const uint64_t* keys, uint64_t n, uint32_t parts, uint64_t* out_keys,
                           uint32_t* out_pos, uint64_t* d_counts, void* ws, hipStream_t stream);

// chunk-of-`chunk` emulation; *d_created accumulates (zero it first).
hipError_t group_chunked(const uint32_t* rep, uint64_t n, uint32_t chunk, uint32_t* rep_chunked,
                         uint64_t* d_created, hipStream_t stream);

}  // namespace sdcas
