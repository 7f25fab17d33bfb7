// thumb.hip — the cas_id string consumers: the thumbnail shard
// directory, thumb key and thumbnail path of a cas_id
// (core/src/object/media/thumbnail/shard.rs:10-13, thumbnail/mod.rs:37-41,62-103), on the
// host for one cas_id and as device batches for a whole library's keys.
//
// A cas_id is the 16 lowercase hex chars of the key (cas.rs:61, sd_cas_key_to_hex); the
// shard is its first 3 chars; a thumbnail lives at
//   <data_dir>/thumbnails/<library_id | "ephemeral">/<shard>/<cas_id>.webp
// Batch layout: one fixed-width record per key, `stride` bytes (a multiple of 16), the
// path NUL-padded — each lane builds 16 consecutive output bytes of the batch, so the
// stores are fully coalesced dwordx4 (byte work: the bound is the HBM write of the records).
// The shared prefix ("<data_dir>/thumbnails/<kind>/") is passed by value in the kernel
// arguments and staged in LDS once per workgroup.
#include <string.h>

#include "ctx_internal.h"

namespace {

constexpr char kThumbDir[] = "thumbnails";  // THUMBNAIL_CACHE_DIR_NAME, mod.rs:37
constexpr char kEphemeral[] = "ephemeral";  // EPHEMERAL_DIR, mod.rs:41
constexpr char kExt[] = ".webp";            // "." + WEBP_EXTENSION, mod.rs:40
constexpr uint32_t kTail = 3 + 1 + 16 + 5;  // shard '/' cas_id ".webp"
constexpr uint32_t kMaxPrefix = 1024;  // the prefix travels in the kernel arguments
constexpr uint32_t kMaxStride = 2048;
constexpr uint32_t kThreads = 256;

__device__ __forceinline__ uint32_t hex_digit(uint64_t key, uint32_t i) {  // i-th of 16
  const uint32_t v = (uint32_t)(key >> (60 - 4 * i)) & 15u;
  return v < 10 ? '0' + v : 'a' + (v - 10);
}

}  // namespace

struct ThumbPrefix {
  uint8_t bytes[kMaxPrefix];
};

// The 16 hex chars of a key as 4 little-endian words (char 4i+j = byte j of word i): each
// 16-bit chunk spread to one nibble per byte, then SWAR ascii ('0' + n, +39 for a-f).
__device__ __forceinline__ uint32_t hex_word(uint64_t key, int i) {
  const uint32_t c = (uint32_t)(key >> (48 - 16 * i)) & 0xFFFFu;
  const uint32_t v = (c >> 12) | (((c >> 8) & 15u) << 8) | (((c >> 4) & 15u) << 16) | ((c & 15u) << 24);
  return v + 0x30303030u + (((v + 0x06060606u) >> 4) & 0x01010101u) * 39u;
}

// word (4 bytes at record offset o, o % 4 == 0) of prefix ‖ tail ‖ zeros, where the tail is
// shard '/' cas_id ".webp" = 25 bytes, held as 8 words tw[0..7] (tw[7] = 0)
__device__ __forceinline__ uint32_t tail_word(const uint32_t (&tw)[8], int d) {  // d = o - P >= 0
  const int a = d >> 2, sh = (d & 3) * 8;
  uint32_t lo = 0, hi = 0;
#pragma unroll
  for (int j = 0; j < 8; ++j) {  // select, not a dynamically indexed (scratch) array
    lo = a == j ? tw[j] : lo;
    hi = a + 1 == j ? tw[j] : hi;
  }
  return sh ? (lo >> sh) | (hi << (32 - sh)) : lo;
}

extern "C" __global__ void __launch_bounds__(kThreads)
sd_thumb_paths(const uint64_t* __restrict__ keys, uint64_t n, uint32_t stride,
               const ThumbPrefix prefix, uint32_t plen, uint4* __restrict__ out) {
  __shared__ uint4 pre4[kMaxPrefix / 16];  // the prefix as 16-B quads (zero-padded)
  uint8_t* pre = reinterpret_cast<uint8_t*>(pre4);
  const uint32_t* prew = reinterpret_cast<const uint32_t*>(pre4);
  for (uint32_t i = threadIdx.x; i < kMaxPrefix; i += kThreads) pre[i] = i < plen ? prefix.bytes[i] : 0;
  __syncthreads();
  const uint32_t q_per = stride >> 4;  // 16-B quads per record
  const uint64_t total = n * q_per;
  for (uint64_t g = (uint64_t)blockIdx.x * kThreads + threadIdx.x; g < total;
       g += (uint64_t)gridDim.x * kThreads) {
    // 32-bit index math while the batch has < 2^32 quads (always, in practice)
    const uint64_t r = total < (1ull << 32) ? (uint32_t)g / q_per : g / q_per;
    const uint32_t o0 = (uint32_t)(g - r * q_per) << 4;
    uint4 qd;
    if (o0 + 16 <= plen) {
      qd = pre4[o0 >> 4];  // a quad wholly inside the prefix: one LDS read
    } else if (o0 >= plen + kTail) {
      qd = make_uint4(0u, 0u, 0u, 0u);  // NUL padding
    } else {  // the 2-3 quads holding the end of the prefix and the 25-byte tail
      const uint64_t key = keys[r];
      uint32_t tw[8];
      tw[1] = hex_word(key, 0);
      tw[2] = hex_word(key, 1);
      tw[3] = hex_word(key, 2);
      tw[4] = hex_word(key, 3);
      tw[0] = (tw[1] & 0x00FFFFFFu) | ((uint32_t)'/' << 24);  // shard + '/'
      tw[5] = 0x6265772Eu;                                     // ".web"
      tw[6] = (uint32_t)'p';
      tw[7] = 0u;
      uint32_t w[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int o = (int)o0 + 4 * k, d = o - (int)plen;
        if (d >= 0) {
          w[k] = d < (int)kTail ? tail_word(tw, d) : 0u;
        } else if (d <= -4) {
          w[k] = prew[o >> 2];
        } else {  // -3..-1: the prefix's last bytes, then the tail's first
          const int keep = -d;  // prefix bytes in this word
          w[k] = (prew[o >> 2] & ((1u << (8 * keep)) - 1u)) | (tw[0] << (8 * keep));
        }
      }
      qd = make_uint4(w[0], w[1], w[2], w[3]);
    }
    out[g] = qd;
  }
}

// the cas_id column of a batch: 16 hex chars per key, no NUL (one dwordx4 store per key)
extern "C" __global__ void __launch_bounds__(kThreads)
sd_keys_to_hex(const uint64_t* __restrict__ keys, uint64_t n, uint4* __restrict__ out) {
  for (uint64_t i = (uint64_t)blockIdx.x * kThreads + threadIdx.x; i < n;
       i += (uint64_t)gridDim.x * kThreads) {
    const uint64_t key = keys[i];
    uint32_t w[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      uint32_t v = 0;
#pragma unroll
      for (int b = 0; b < 4; ++b) v |= hex_digit(key, 4 * k + b) << (8 * b);
      w[k] = v;
    }
    out[i] = make_uint4(w[0], w[1], w[2], w[3]);
  }
}

namespace {

uint32_t grid_for(uint64_t items) {
  const uint64_t b = (items + kThreads - 1) / kThreads;
  return (uint32_t)(b < 8192 ? (b ? b : 1) : 8192);  // grid-stride above 2M items
}

// snprintf-like: write s into out[pos..cap) as far as it fits, return the new length
size_t put(char* out, size_t cap, size_t pos, const char* s, size_t len) {
  for (size_t i = 0; i < len; ++i, ++pos)
    if (out && pos + 1 < cap) out[pos] = s[i];
  return pos;
}

}  // namespace

extern "C" {

void sd_cas_shard_hex(uint64_t key, char out[4]) {
  char hex[17];
  sd_cas_key_to_hex(key, hex);
  out[0] = hex[0];
  out[1] = hex[1];
  out[2] = hex[2];
  out[3] = 0;
}

int64_t sd_cas_thumbnail_path(const char* data_dir, const char* library_id, uint64_t key,
                              char* out, size_t cap) {
  if (!data_dir || (cap && !out)) return SD_CAS_EINVAL;
  char hex[17];
  sd_cas_key_to_hex(key, hex);
  const char* kind = library_id ? library_id : kEphemeral;
  const size_t ld = strlen(data_dir);
  size_t pos = put(out, cap, 0, data_dir, ld);
  // PathBuf::push: a '/' between components unless the base is empty or already ends in one
  if (ld && data_dir[ld - 1] != '/') pos = put(out, cap, pos, "/", 1);
  pos = put(out, cap, pos, kThumbDir, sizeof(kThumbDir) - 1);
  pos = put(out, cap, pos, "/", 1);
  pos = put(out, cap, pos, kind, strlen(kind));
  pos = put(out, cap, pos, "/", 1);
  pos = put(out, cap, pos, hex, 3);
  pos = put(out, cap, pos, "/", 1);
  pos = put(out, cap, pos, hex, 16);
  pos = put(out, cap, pos, kExt, sizeof(kExt) - 1);
  if (cap) out[pos < cap ? pos : cap - 1] = 0;
  return (int64_t)pos;
}

int64_t sd_cas_thumb_key(const char* library_id, uint64_t key, char* out, size_t cap) {
  if (cap && !out) return SD_CAS_EINVAL;
  char hex[17];
  sd_cas_key_to_hex(key, hex);
  const char* kind = library_id ? library_id : kEphemeral;
  const size_t lk = strlen(kind), need = lk + 1 + 4 + 17;
  if (need > cap) return (int64_t)need;
  memcpy(out, kind, lk + 1);
  memcpy(out + lk + 1, hex, 3);
  out[lk + 4] = 0;
  memcpy(out + lk + 5, hex, 17);
  return (int64_t)need;
}

int sd_cas_keys_to_hex_dev(sd_cas_ctx* c, const uint64_t* d_keys, size_t n, char* d_out,
                           void* stream) {
  if (!c) return SD_CAS_EINVAL;
  if (n == 0) return SD_CAS_OK;
  if (!d_keys || !d_out || ((uintptr_t)d_out & 15) || ((uintptr_t)d_keys & 7))
    return sd_fail(c, SD_CAS_EINVAL, "keys_to_hex: bad arguments");
  hipStream_t s = sd_pick(c, stream);
  sd_keys_to_hex<<<grid_for(n), kThreads, 0, s>>>(d_keys, n, (uint4*)d_out);
  HIP_TRY(c, hipGetLastError());
  return SD_CAS_OK;
}

int sd_cas_thumbnail_paths_dev(sd_cas_ctx* c, const uint64_t* d_keys, size_t n,
                               const char* prefix, uint32_t stride, char* d_out, void* stream) {
  if (!c) return SD_CAS_EINVAL;
  const size_t plen = prefix ? strlen(prefix) : 0;
  if (!prefix || plen > kMaxPrefix || stride == 0 || (stride & 15) || stride > kMaxStride ||
      plen + kTail + 1 > stride)
    return sd_fail(c, SD_CAS_EINVAL,
                   "thumbnail_paths: prefix of %zu B (<= %u) + %u B + NUL must fit a stride "
                   "(%u) that is a multiple of 16 <= %u", plen, kMaxPrefix, kTail, stride,
                   kMaxStride);
  if (n == 0) return SD_CAS_OK;
  if (!d_keys || !d_out || ((uintptr_t)d_out & 15) || ((uintptr_t)d_keys & 7))
    return sd_fail(c, SD_CAS_EINVAL, "thumbnail_paths: bad pointers");
  ThumbPrefix pre{};
  memcpy(pre.bytes, prefix, plen);
  const uint64_t quads = (uint64_t)n * (stride >> 4);
  sd_thumb_paths<<<grid_for(quads), kThreads, 0, sd_pick(c, stream)>>>(d_keys, n, stride, pre,
                                                                       (uint32_t)plen,
                                                                       (uint4*)d_out);
  HIP_TRY(c, hipGetLastError());
  return SD_CAS_OK;
}

}  // extern "C"
