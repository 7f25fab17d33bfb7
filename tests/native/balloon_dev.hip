// balloon_dev.hip — TEST INFRASTRUCTURE: the reference's Balloon-BLAKE3 password hash run on
// the GPU with the product's device BLAKE3 (spacedrive_amd/csrc/blake3_device.hpp: the
// compression every kernel uses — message schedule, G rotations, flags, feed-forward), so
// that device code reproduces the reference's own known answers,
// crates/crypto/src/keys/hashing.rs:180-208 (HASH_B3BALLOON[_WITH_SECRET]_EXPECTED), not only
// the oracle's outputs.  The construction is oracle/balloon_ref.c's (Balloon, ePrint 2016/027
// §3.1, delta 3; the secret in the first block's and the index hashes).  Each job is one
// inherently sequential chain of ~2.75 M BLAKE3 hashes (s_cost 131,072, t_cost 2) on one lane;
// jobs run side by side in separate workgroups, and the chain is cut into launches of <= 8,192
// blocks so no single kernel runs long.  Built by tests/test_gpu_parity.py into
// tests/native/libballoon_dev.so (git-ignored); nothing in the product loads it.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../spacedrive_amd/csrc/blake3_device.hpp"

using namespace sdcas;

struct Job {
  const uint8_t* pwd;
  const uint8_t* salt;
  const uint8_t* secret;
  uint32_t pwd_len, salt_len, secret_len;
  uint8_t* buf;     // s_cost x 32 B
  uint64_t* cnt;    // the chain's counter between launches
};

__device__ void put(uint8_t* msg, uint32_t& n, const uint8_t* p, uint32_t len) {
  for (uint32_t i = 0; i < len; i++) msg[n++] = p[i];
}
__device__ void put64(uint8_t* msg, uint32_t& n, uint64_t v) {
  for (int i = 0; i < 8; i++) msg[n++] = (uint8_t)(v >> (8 * i));
}

// BLAKE3 of msg[0, len) (len <= 128: one chunk, 1-2 blocks) -> out (32 B, little-endian words)
__device__ void hash_msg(const uint8_t* msg, uint32_t len, uint8_t* out) {
  uint32_t cv[8];
  set_iv(cv);
  const uint32_t nb = len ? (len + 63) / 64 : 1;
  for (uint32_t b = 0; b < nb; b++) {
    uint32_t m[16];
#pragma unroll
    for (int w = 0; w < 16; w++) {
      uint32_t v = 0;
      for (int k = 3; k >= 0; k--) {
        const uint32_t i = b * 64 + 4 * w + k;
        v = (v << 8) | (i < len ? msg[i] : 0u);
      }
      m[w] = v;
    }
    const uint32_t blen = len - b * 64 < 64 ? len - b * 64 : 64;
    const uint32_t flags = (b == 0 ? CHUNK_START : 0u) | (b + 1 == nb ? (CHUNK_END | ROOT) : 0u);
    compress(cv, m, 0u, 0u, blen, flags);
  }
  for (int w = 0; w < 8; w++)
    for (int k = 0; k < 4; k++) out[4 * w + k] = (uint8_t)(cv[w] >> (8 * k));
}

// Step 1 for job blockIdx.x: buf[0] = H(cnt++, pwd, salt[, secret]); buf[m] = H(cnt++, buf[m-1])
extern "C" __global__ void __launch_bounds__(64) balloon_expand(const Job* jobs, uint64_t s_cost) {
  if (threadIdx.x) return;
  const Job j = jobs[blockIdx.x];
  __shared__ uint8_t msg[160];
  uint64_t cnt = 0;
  uint32_t n = 0;
  put64(msg, n, cnt++);
  put(msg, n, j.pwd, j.pwd_len);
  put(msg, n, j.salt, j.salt_len);
  put(msg, n, j.secret, j.secret_len);
  hash_msg(msg, n, j.buf);
  for (uint64_t m = 1; m < s_cost; m++) {
    n = 0;
    put64(msg, n, cnt++);
    put(msg, n, j.buf + 32 * (m - 1), 32);
    hash_msg(msg, n, j.buf + 32 * m);
  }
  *j.cnt = cnt;
}

// Step 2 for blocks [m0, m1) of round t
extern "C" __global__ void __launch_bounds__(64) balloon_mix(const Job* jobs, uint64_t s_cost,
                                                           uint64_t t, uint64_t m0, uint64_t m1) {
  if (threadIdx.x) return;
  const Job j = jobs[blockIdx.x];
  __shared__ uint8_t msg[160];
  __shared__ uint8_t idx[32], oth[32];
  uint64_t cnt = *j.cnt;
  for (uint64_t m = m0; m < m1; m++) {
    uint8_t* cur = j.buf + 32 * m;
    const uint8_t* prev = j.buf + 32 * (m ? m - 1 : s_cost - 1);
    uint32_t n = 0;
    put64(msg, n, cnt++);
    put(msg, n, prev, 32);
    put(msg, n, cur, 32);
    hash_msg(msg, n, cur);
    for (uint64_t i = 0; i < 3; i++) {
      n = 0;
      put64(msg, n, t);
      put64(msg, n, m);
      put64(msg, n, i);
      hash_msg(msg, n, idx);
      n = 0;
      put64(msg, n, cnt++);
      put(msg, n, j.salt, j.salt_len);
      put(msg, n, j.secret, j.secret_len);
      put(msg, n, idx, 32);
      hash_msg(msg, n, oth);
      uint64_t r = 0;  // the 256-bit little-endian integer mod s_cost (r < s_cost < 2^56)
      for (int k = 31; k >= 0; k--) r = ((r << 8) | oth[k]) % s_cost;
      n = 0;
      put64(msg, n, cnt++);
      put(msg, n, cur, 32);
      put(msg, n, j.buf + 32 * r, 32);
      hash_msg(msg, n, cur);
    }
  }
  *j.cnt = cnt;
}

#define TRY(x) do { if ((x) != hipSuccess) return -1; } while (0)

// njobs chains of one (pwd, salt) with per-job secrets (secret_lens[j] = 0: none); out: 32 B
// per job.  Returns 0, or -1 on a HIP failure.
extern "C" int balloon_dev_run(const uint8_t* pwd, uint32_t pwd_len, const uint8_t* salt,
                               uint32_t salt_len, const uint8_t* const* secrets,
                               const uint32_t* secret_lens, int njobs, uint64_t s_cost,
                               uint64_t t_cost, uint8_t* out) {
  if (njobs < 1 || njobs > 16 || pwd_len > 64 || salt_len > 32 || s_cost == 0 ||
      s_cost >= (1ull << 56))
    return -1;
  uint8_t* d_in;
  Job* d_jobs;
  uint8_t* d_buf;
  uint64_t* d_cnt;
  TRY(hipMalloc(&d_in, 256 * (size_t)njobs));
  TRY(hipMalloc(&d_jobs, sizeof(Job) * njobs));
  TRY(hipMalloc(&d_buf, 32 * s_cost * njobs));
  TRY(hipMalloc(&d_cnt, 8 * njobs));
  Job h[16];
  for (int k = 0; k < njobs; k++) {
    uint8_t tmp[256] = {0};
    for (uint32_t i = 0; i < pwd_len; i++) tmp[i] = pwd[i];
    for (uint32_t i = 0; i < salt_len; i++) tmp[64 + i] = salt[i];
    const uint32_t sl = secret_lens[k] > 64 ? 64 : secret_lens[k];
    for (uint32_t i = 0; i < sl; i++) tmp[128 + i] = secrets[k][i];
    TRY(hipMemcpy(d_in + 256 * k, tmp, 256, hipMemcpyHostToDevice));
    h[k] = Job{d_in + 256 * k, d_in + 256 * k + 64, d_in + 256 * k + 128, pwd_len, salt_len, sl,
               d_buf + 32 * s_cost * k, d_cnt + k};
  }
  TRY(hipMemcpy(d_jobs, h, sizeof(Job) * njobs, hipMemcpyHostToDevice));
  balloon_expand<<<njobs, 64>>>(d_jobs, s_cost);
  TRY(hipGetLastError());
  const uint64_t piece = 8192;
  for (uint64_t t = 0; t < t_cost; t++)
    for (uint64_t m0 = 0; m0 < s_cost; m0 += piece) {
      balloon_mix<<<njobs, 64>>>(d_jobs, s_cost, t, m0, m0 + piece < s_cost ? m0 + piece : s_cost);
      TRY(hipGetLastError());
    }
  TRY(hipDeviceSynchronize());
  for (int k = 0; k < njobs; k++)
    TRY(hipMemcpy(out + 32 * k, d_buf + 32 * s_cost * k + 32 * (s_cost - 1), 32, hipMemcpyDeviceToHost));
  TRY(hipFree(d_in));
  TRY(hipFree(d_jobs));
  TRY(hipFree(d_buf));
  TRY(hipFree(d_cnt));
  return 0;
}
