// sd_checksum.h — host launchers for the validator tree hash (checksum.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace sdcas {

size_t checksum_workspace_bytes(uint64_t len);

// BLAKE3 tree over data[0, len) whose first chunk has global index chunk0.
// root == true: d_out8 = the 32-byte digest (this buffer is the whole input).
// root == false: d_out8 = the subtree CV (len must then be a power-of-two multiple of
// 1 KiB aligned at chunk0, i.e. a complete left subtree, for the result to be usable).
hipError_t checksum_device(const uint8_t* data, uint64_t len, uint64_t chunk0, bool root,
                           uint32_t* d_out8, void* ws, hipStream_t s);

// Root digest over `cnt` subtree CVs (level-wise; ROOT on the final parent).
hipError_t reduce_cvs_device(const uint32_t* d_cvs, uint64_t cnt, uint32_t* d_out8, void* ws,
                             hipStream_t s);

// Many buffers in one launch chain: buffer i = arena[offs[i], offs[i] + lens[i]) (16-B
// aligned, readable to the 16-B round-up), d_digests[8 i ..] = its 32-byte digest.
// arena_bytes bounds every buffer's end (sizes the CV list); a buffer over 64 GiB sets *d_bad.
// n <= 2^24.  ws: checksum_batch_workspace_bytes(n, arena_bytes).
size_t checksum_batch_workspace_bytes(uint64_t n, uint64_t arena_bytes);
// d_ol[0] = 0, d_ol[1] = len, *d_bad = 0 (the one-buffer batch of sd_cas_checksum_dev)
hipError_t checksum_single_setup(uint64_t* d_ol, uint64_t len, uint32_t* d_bad, hipStream_t s);
hipError_t checksum_batch_device(const uint8_t* arena, uint64_t arena_bytes, const uint64_t* offs,
                                 const uint64_t* lens, uint64_t n, uint32_t* d_digests,
                                 uint32_t* d_bad, void* ws, hipStream_t s);

}  // namespace sdcas
