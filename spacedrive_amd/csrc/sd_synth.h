// sd_synth.h — synthetic-input launchers (synth.hip); definitions mirror oracle/cas_ref.c.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace sdcas {

enum : uint32_t { SYNTH_SAMPLED = 0, SYNTH_SMALL = 1 };

__host__ __device__ uint64_t synth_root(uint64_t seed, uint64_t f, uint32_t dup_permille);
__host__ __device__ uint64_t synth_size(uint64_t seed, uint64_t root, uint32_t kind);

hipError_t synth_sampled(uint64_t seed, uint64_t file0, uint64_t n, uint32_t dup_permille,
                         uint8_t* content, uint64_t stride, uint64_t* sizes, hipStream_t s);
hipError_t synth_small_sizes(uint64_t seed, uint64_t file0, uint64_t n, uint32_t dup_permille,
                             uint64_t* sizes, uint32_t* lens, hipStream_t s);
hipError_t synth_small_content(uint64_t seed, uint64_t file0, uint64_t n, uint32_t dup_permille,
                               const uint64_t* offs, const uint32_t* lens, uint8_t* arena,
                               hipStream_t s);
// bytes [byte_off, byte_off + len) of file `file`'s stream (byte_off, out 8-B aligned; the
// last word is written whole: out must hold the 8-B round-up of len)
hipError_t synth_stream(uint64_t seed, uint64_t file, uint64_t byte_off, uint64_t len,
                        uint8_t* out, hipStream_t s);
hipError_t synth_roots(uint64_t seed, uint64_t file0, uint64_t n, uint32_t dup_permille,
                       uint64_t* roots, hipStream_t s);

}  // namespace sdcas
