// sd_mix.h — the grouping's key mix and coarse-bucket function, shared by the grouping
// kernels (group_hash.hip) and the hash kernels that partition their own output
// (cas_hash.hip, the fused hash + group chain).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace sdcas {

// splitmix64 finalizer: a bijection on u64, so distinct keys stay distinct
__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// The fused chain's coarse buckets: the top REGION_BITS bits of the mixed key, each with a
// fixed-capacity region of rows (mixed key u64, file u32) written by the hash kernel.
// 2^8 regions: one 1,024-lane table workgroup per CU over ~5,100 keys.  SD_REGION_BITS=9 (two
// 512-lane workgroups per CU over ~2,560 keys each) measured slower: 0.0224 vs 0.0213 ms at
// 1.31M keys, K1G unchanged (profiles/r03b_group_ab/README.md)
#ifndef SD_REGION_BITS
#define SD_REGION_BITS 8
#endif
constexpr uint32_t REGION_BITS = SD_REGION_BITS;
constexpr uint32_t REGIONS = 1u << REGION_BITS;
// A region set's persistent counters (zero between calls): REGIONS row cursors, then the
// spill count (rows past their region's capacity, appended to the set's spill list), the
// count of full regions and the tables' count of full regions done (the last one re-zeroes
// the three)
constexpr uint32_t REGION_SPILL_WORD = REGIONS;
constexpr uint32_t REGION_SET_WORDS = REGIONS + 32;

}  // namespace sdcas
