// synth.hip — on-device synthetic inputs for benches and GPU parity tests.
//
// Same counter-based splitmix64 definitions as oracle/cas_ref.c (orc_mix64 /
// orc_file_key / orc_fill_content) and oracle/pyoracle.py, so the CPU oracle can
// regenerate any file the GPU hashes.  Duplicate content (BASELINE config 4) follows a
// chain to the root content id: file f duplicates a uniformly chosen earlier file with
// probability dup_permille/1000.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "sd_synth.h"

namespace sdcas {

constexpr uint64_t GAMMA = 0x9E3779B97F4A7C15ull;

__host__ __device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
__host__ __device__ __forceinline__ uint64_t file_key(uint64_t seed, uint64_t f) {
  return mix64(mix64(seed) + f * GAMMA);
}
__host__ __device__ uint64_t synth_root(uint64_t seed, uint64_t f, uint32_t dup_permille) {
  while (f > 0 && dup_permille) {
    const uint64_t h = mix64(file_key(seed ^ 0xD0D0D0D0D0D0D0D0ull, f));
    if ((h % 1000u) >= dup_permille) break;
    f = (h >> 20) % f;
  }
  return f;
}
__host__ __device__ uint64_t synth_size(uint64_t seed, uint64_t root, uint32_t kind) {
  const uint64_t h = mix64(file_key(seed, root) ^ 0x53495A4553495A45ull);
  if (kind == SYNTH_SAMPLED)  // (102,400, 2^32]
    return 102401ull + h % ((1ull << 32) - 102400ull);
  return 1ull + h % 102400ull;  // whole-file path: [1, 102,400]
}

// content of `n` sampled files (57,344 B each) at `stride`; 16 B per thread per step
extern "C" __global__ void __launch_bounds__(256)
sd_synth_sampled(uint64_t seed, uint64_t file0, uint64_t n, uint32_t dup_permille,
                 uint8_t* __restrict__ content, uint64_t stride, uint64_t* __restrict__ sizes) {
  constexpr uint64_t QPF = 57344 / 16;  // quads per file
  const uint64_t total = n * QPF;
  for (uint64_t q = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; q < total;
       q += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t fl = q / QPF, w = (q % QPF) * 2;
    const uint64_t root = synth_root(seed, file0 + fl, dup_permille);
    const uint64_t key = file_key(seed, root);
    const uint64_t a = mix64(key + (w + 1) * GAMMA), b = mix64(key + (w + 2) * GAMMA);
    *reinterpret_cast<ulonglong2*>(content + fl * stride + (q % QPF) * 16) = make_ulonglong2(a, b);
    if (w == 0) sizes[fl] = synth_size(seed, root, SYNTH_SAMPLED);
  }
}

// whole-file sizes (pass 1): sizes[i], lens[i] = size
extern "C" __global__ void __launch_bounds__(256)
sd_synth_small_sizes(uint64_t seed, uint64_t file0, uint64_t n, uint32_t dup_permille,
                     uint64_t* __restrict__ sizes, uint32_t* __restrict__ lens) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t root = synth_root(seed, file0 + i, dup_permille);
  const uint64_t s = synth_size(seed, root, SYNTH_SMALL);
  sizes[i] = s;
  lens[i] = (uint32_t)s;
}

// whole-file content (pass 2, after offsets = exclusive scan of 16-B-rounded lens):
// one workgroup per file, 16 B per thread per step (tail bytes past len left as is)
extern "C" __global__ void __launch_bounds__(256)
sd_synth_small_content(uint64_t seed, uint64_t file0, uint64_t n, uint32_t dup_permille,
                       const uint64_t* __restrict__ offs, const uint32_t* __restrict__ lens,
                       uint8_t* __restrict__ arena) {
  for (uint64_t i = blockIdx.x; i < n; i += gridDim.x) {
    const uint64_t root = synth_root(seed, file0 + i, dup_permille);
    const uint64_t key = file_key(seed, root);
    const uint32_t nq = (lens[i] + 15u) >> 4;
    uint8_t* dst = arena + offs[i];
    for (uint32_t q = threadIdx.x; q < nq; q += blockDim.x) {
      const uint64_t w = (uint64_t)q * 2;
      *reinterpret_cast<ulonglong2*>(dst + (uint64_t)q * 16) =
          make_ulonglong2(mix64(key + (w + 1) * GAMMA), mix64(key + (w + 2) * GAMMA));
    }
  }
}

extern "C" __global__ void __launch_bounds__(256)
sd_synth_roots(uint64_t seed, uint64_t file0, uint64_t n, uint32_t dup_permille,
               uint64_t* __restrict__ roots) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) roots[i] = synth_root(seed, file0 + i, dup_permille);
}

// bytes [8*w0, 8*(w0+nw)) of file `file`'s content stream (the validator's multi-GiB files)
extern "C" __global__ void __launch_bounds__(256)
sd_synth_stream(uint64_t seed, uint64_t file, uint64_t w0, uint64_t nw, uint64_t* __restrict__ out) {
  const uint64_t key = file_key(seed, file);
  for (uint64_t w = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; w < nw;
       w += (uint64_t)gridDim.x * blockDim.x)
    out[w] = mix64(key + (w0 + w + 1) * GAMMA);
}

hipError_t synth_stream(uint64_t seed, uint64_t file, uint64_t byte_off, uint64_t len,
                        uint8_t* out, hipStream_t s) {
  if (len == 0) return hipSuccess;
  if ((byte_off & 7) || ((uintptr_t)out & 7)) return hipErrorInvalidValue;
  sd_synth_stream<<<256 * 64, 256, 0, s>>>(seed, file, byte_off >> 3, (len + 7) >> 3,
                                           reinterpret_cast<uint64_t*>(out));
  return hipGetLastError();
}

hipError_t synth_sampled(uint64_t seed, uint64_t file0, uint64_t n, uint32_t dup_permille,
                         uint8_t* content, uint64_t stride, uint64_t* sizes, hipStream_t s) {
  if (n == 0) return hipSuccess;
  sd_synth_sampled<<<256 * 32, 256, 0, s>>>(seed, file0, n, dup_permille, content, stride, sizes);
  return hipGetLastError();
}

hipError_t synth_small_sizes(uint64_t seed, uint64_t file0, uint64_t n, uint32_t dup_permille,
                             uint64_t* sizes, uint32_t* lens, hipStream_t s) {
  if (n == 0) return hipSuccess;
  sd_synth_small_sizes<<<(uint32_t)((n + 255) / 256), 256, 0, s>>>(seed, file0, n, dup_permille,
                                                                   sizes, lens);
  return hipGetLastError();
}

hipError_t synth_small_content(uint64_t seed, uint64_t file0, uint64_t n, uint32_t dup_permille,
                               const uint64_t* offs, const uint32_t* lens, uint8_t* arena,
                               hipStream_t s) {
  if (n == 0) return hipSuccess;
  sd_synth_small_content<<<256 * 16, 256, 0, s>>>(seed, file0, n, dup_permille, offs, lens, arena);
  return hipGetLastError();
}

hipError_t synth_roots(uint64_t seed, uint64_t file0, uint64_t n, uint32_t dup_permille,
                       uint64_t* roots, hipStream_t s) {
  if (n == 0) return hipSuccess;
  sd_synth_roots<<<(uint32_t)((n + 255) / 256), 256, 0, s>>>(seed, file0, n, dup_permille, roots);
  return hipGetLastError();
}

}  // namespace sdcas
