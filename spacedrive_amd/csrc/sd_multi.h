// sd_multi.h — launchers for multi.hip (single-process multi-device grouping).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace sdcas {

hipError_t multi_splits(const uint64_t* skeys, uint64_t n, uint32_t G, uint64_t* splits,
                        hipStream_t s);
hipError_t multi_gidx(const uint32_t* sidx, uint64_t n, uint64_t file0, uint64_t* gidx,
                      hipStream_t s);
hipError_t multi_gather(const uint32_t* rep_pos, const uint64_t* ridx, uint64_t m, uint64_t* out,
                        hipStream_t s);
hipError_t multi_scatter(const uint32_t* sidx, const uint64_t* back, uint64_t n, uint64_t* rep,
                         hipStream_t s);

// the per-process RCCL exchange (spacedrive_amd/shard.py): 12-byte (key, u32 idx) rows
hipError_t exch_pack(const uint64_t* keys, const uint32_t* pos, uint64_t n, uint64_t file0,
                     uint32_t* rows, hipStream_t s);
hipError_t exch_split(const uint32_t* rows, uint64_t m, uint64_t* keys, uint32_t* vals,
                      hipStream_t s);
hipError_t exch_unpack(const uint32_t* back, const uint32_t* pos, uint64_t n, uint64_t* rep,
                       hipStream_t s);
// fixed-capacity variants (G <= 1024 blocks of cap rows + G spill blocks of spill rows)
hipError_t exch_pack_fixed(const uint64_t* keys, const uint32_t* pos, const uint64_t* counts,
                           uint32_t G, uint64_t cap, uint64_t spill, uint64_t file0, uint32_t* rows,
                           uint32_t* srows, uint32_t* overflow, hipStream_t s);
hipError_t exch_split_fixed(const uint32_t* rows, uint64_t m, uint64_t sentinel, uint64_t* keys,
                            uint32_t* vals, uint64_t* sentinel_rows, hipStream_t s);
hipError_t exch_unpack_fixed(const uint32_t* back, const uint32_t* sback, const uint32_t* pos,
                             const uint64_t* counts, uint32_t G, uint64_t cap, uint64_t spill,
                             uint64_t* rep, hipStream_t s);

}  // namespace sdcas
