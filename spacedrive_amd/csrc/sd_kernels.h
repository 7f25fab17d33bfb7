// sd_kernels.h — internal constants shared by the HIP kernels and the C-ABI layer.
#pragma once
#include <stdint.h>

namespace sdcas {

// core/src/object/cas.rs:10-15
constexpr uint64_t SAMPLE_COUNT = 4;
constexpr uint64_t SAMPLE_SIZE = 1024 * 10;
constexpr uint64_t HEADER_OR_FOOTER_SIZE = 1024 * 8;
constexpr uint64_t MINIMUM_FILE_SIZE = 1024 * 100;
constexpr uint32_t SAMPLED_CONTENT_LEN =
    (uint32_t)(2 * HEADER_OR_FOOTER_SIZE + SAMPLE_COUNT * SAMPLE_SIZE);  // 57,344
// cas.rs:18 const_assert!((HEADER_OR_FOOTER_SIZE * 2 + SAMPLE_COUNT * SAMPLE_SIZE) < MINIMUM_FILE_SIZE)
static_assert(2 * HEADER_OR_FOOTER_SIZE + SAMPLE_COUNT * SAMPLE_SIZE < MINIMUM_FILE_SIZE, "cas.rs:18");
// cas.rs:21 const_assert!(SAMPLE_SIZE > HEADER_OR_FOOTER_SIZE)
static_assert(SAMPLE_SIZE > HEADER_OR_FOOTER_SIZE, "cas.rs:21");

// The packed (whole-file) kernel keeps a 6-deep CV stack: messages of <= 104 chunks
// (a whole file is <= 102,400 + 8 bytes = 101 chunks).
constexpr uint32_t MAX_PACKED_CONTENT_LEN = 104u * 1024u - 8u;

}  // namespace sdcas

#include <hip/hip_runtime.h>
namespace sdcas {
// cus = the device's CU count: batches of fewer 512-lane workgroups than CUs take the
// 256-lane grid (one wave per SIMD instead of half the CUs at two)
hipError_t hash_sampled(const uint8_t* content, uint64_t stride, const uint64_t* sizes,
                        uint64_t n, uint64_t* keys, hipStream_t s, uint32_t cus);
// K1G: K1 + the grouping partition in its epilogue (cas_hash.hip): keys, rep[f] = f, and
// each key's (mix64(key), f) row in the fixed-capacity region of its coarse bucket
// (rkeys/rfile [REGIONS][cap], cursor [REGIONS] zero on entry); *overflow |= 1 when a region
// is full; *objects = 0 (the bucket tables count).
hipError_t hash_sampled_regions(const uint8_t* content, uint64_t stride, const uint64_t* sizes,
                                uint64_t n, uint64_t* keys, uint32_t* rep, uint64_t* rkeys,
                                uint32_t* rfile, uint32_t* cursor, uint64_t cap, uint64_t* spill_keys,
                                uint32_t* spill_file, uint32_t* overflow, uint64_t* objects,
                                hipStream_t s, uint32_t cus);
// pinned host -> device copy by a kernel (16-B aligned; else hipMemcpyAsync)
hipError_t pull_host(void* dst, const void* src, uint64_t bytes, hipStream_t s);
hipError_t hash_packed(const uint8_t* arena, const uint64_t* offs, const uint32_t* lens,
                       const uint64_t* sizes, const uint32_t* order, uint64_t n, uint64_t* keys,
                       hipStream_t s);
hipError_t length_keys(const uint32_t* lens, uint64_t n, uint64_t* out, hipStream_t s);
// K1L: a file per `seg`-lane segment (64: one wave per file, lane per chunk; 16: four files
// per wave, 4+ chunks per lane) (offs == nullptr: strided, fixed_len bytes each)
hipError_t hash_chunkpar(const uint8_t* arena, const uint64_t* offs, uint64_t stride,
                         const uint32_t* lens, uint32_t fixed_len, const uint64_t* sizes,
                         uint64_t n, uint64_t* keys, int seg, hipStream_t s,
                         const uint32_t* order = nullptr);
int length_key_bits(uint64_t n);  // significant bits of the length_keys sort key
}  // namespace sdcas
