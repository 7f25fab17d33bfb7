// sd_links.h — launchers of the Object-link emission kernels (links.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

// row states / actions / sentinels: the same values as include/sd_hip_cas.h
#define SD_LINKS_HASHED 0
#define SD_LINKS_NO_CAS 1
#define SD_LINKS_ERROR 2
#define SD_LINKS_CREATED 0
#define SD_LINKS_LINKED 1
#define SD_LINKS_DROPPED 2
#define SD_LINKS_NOT_REACHED 3
#define SD_LINKS_EXISTING 4
#define SD_LINKS_NO_STEP 0xFFFFFFFFu
#define SD_LINKS_NO_OBJECT 0xFFFFFFFFu

namespace sdcas {

// A seeded job (Objects that exist before it) tags its rows with ROW_FLAG in the grouping's
// values, so one minimum per key tells an existing Object (< ROW_FLAG: its id) from the
// key's first row (ROW_FLAG | row)
constexpr uint32_t LINKS_ROW_FLAG = 0x80000000u;

// hashed rows -> (hkeys, hrows = row | row_flag) (unordered), other rows -> orphans[] =
// row << 8 | state (state NULL: every row hashed); *d_hcount / *d_ocount (u64, zeroed by the
// caller) = counts
hipError_t links_split(const uint64_t* keys, const uint8_t* state, uint64_t n, uint64_t* hkeys,
                       uint32_t* hrows, uint64_t* d_hcount, uint64_t* orphans, uint64_t* d_ocount,
                       uint32_t row_flag, hipStream_t s);
// rep[hrows[i] & ~row_flag] = minrow[i]
hipError_t links_scatter(const uint32_t* minrow, const uint32_t* hrows, uint64_t m, uint32_t* rep,
                         uint32_t row_flag, hipStream_t s);
// per-row decisions; counts[2k], counts[2k+1] (u32, zeroed by the caller) += created, linked.
// seeded: rep[i] < LINKS_ROW_FLAG is an existing Object's id, else LINKS_ROW_FLAG | first row;
// m > 0 (needs seeded): rows already owning an Object — the sorted event list of
// links_pre_* (ekeys / erows, scan elements T, key filter) and every row's key (keys)
hipError_t links_decide(const uint8_t* state, const uint32_t* rep, uint64_t n,
                        const uint32_t* starts, uint32_t nsteps, uint64_t reached,
                        uint32_t* step_out, uint32_t* object_out, uint8_t* action_out,
                        uint32_t* counts, bool seeded, const uint64_t* keys,
                        const uint64_t* ekeys, const uint32_t* erows, const uint64_t* T,
                        const uint32_t* filter, uint64_t m, uint32_t chunk, hipStream_t s);
// *d_bad (u64, zeroed by the caller) += 1 per wave holding an id >= LINKS_ROW_FLAG (none_ok:
// SD_LINKS_NO_OBJECT allowed)
hipError_t links_check_ids(const uint32_t* ids, uint64_t n, bool none_ok, uint64_t* d_bad,
                           hipStream_t s);
// Rows that already own an Object (pre[r], SD_LINKS_NO_OBJECT = none).  The events (hashed
// rows r < reached with an Object): count -> bcount[pre_blocks(reached)] = the blocks' event
// offsets, *d_total = the number of events (u64, device); emit -> ekeys / erows in row order
// and their keys' bits in `filter` (pre_filter_bytes(), zeroed by the caller); after the
// caller's stable sort of the events by key (skeys / srows), scan -> elem[j] (low 32 bits) =
// the smallest Object over the key's events in steps up to event j's.  tiles:
// segmin_tiles_bytes(m).
size_t pre_blocks(uint64_t n);
size_t pre_filter_bytes();
size_t segmin_tiles_bytes(uint64_t n);
hipError_t links_pre_count(const uint8_t* state, const uint32_t* pre, uint64_t reached,
                           uint32_t* bcount, uint64_t* d_total, hipStream_t s);
hipError_t links_pre_emit(const uint64_t* keys, const uint8_t* state, const uint32_t* pre,
                          uint64_t reached, const uint32_t* boff, uint64_t* ekeys,
                          uint32_t* erows, uint32_t* filter, hipStream_t s);
hipError_t links_pre_scan(const uint64_t* skeys, const uint32_t* srows, const uint32_t* pre,
                          uint64_t m, const uint32_t* starts, uint32_t nsteps, uint64_t* elem,
                          uint64_t* tiles, hipStream_t s);

}  // namespace sdcas
