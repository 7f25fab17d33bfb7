// ubench_gtable.hip — prices a one-level GLOBAL hash table for the Object grouping at small
// n (the bench's 1.31 M keys per GPU), against the partition + LDS-table chain (~0.055 ms):
//   clear  : memset of the table (keys 0, mins 0xFF..)
//   insert : per key one 64-bit CAS (linear probing) + one atomic min, device scope
//   lookup : per key probe to its slot, rep = the slot's min
// Slots are 16 B {u64 mixed key, u32 min, u32 pad} so a probe touches one line.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/ubench_gtable tools/ubench_gtable.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <vector>

#define CHECK(x)                                                                     \
  do {                                                                               \
    hipError_t e = (x);                                                              \
    if (e != hipSuccess) {                                                           \
      fprintf(stderr, "%s: %s (%s:%d)\n", #x, hipGetErrorString(e), __FILE__, __LINE__); \
      exit(1);                                                                       \
    }                                                                                \
  } while (0)

struct Slot {
  unsigned long long key;
  unsigned int min;
  unsigned int pad;
};

__device__ __forceinline__ unsigned long long mix64(unsigned long long z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// keys are nonzero after mixing in this benchmark (the product would route mix == 0 aside)
__global__ void k_insert(const unsigned long long* keys, unsigned n, Slot* t, unsigned mask,
                         unsigned long long* objects) {
  const unsigned i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned fresh = 0;
  if (i < n) {
    const unsigned long long m = mix64(keys[i]);
    unsigned s = (unsigned)m & mask;
    for (;;) {
      unsigned long long cur = __hip_atomic_load(&t[s].key, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (cur == 0) {
        cur = atomicCAS(&t[s].key, 0ull, m);
        if (cur == 0) { fresh = 1; cur = m; }
      }
      if (cur == m) { atomicMin(&t[s].min, i); break; }
      s = (s + 1) & mask;
    }
  }
  // wave-aggregated object count
  const unsigned long long b = __ballot(fresh);
  if ((threadIdx.x & 63) == 0 && b) atomicAdd(objects, (unsigned long long)__popcll(b));
}

__global__ void k_lookup(const unsigned long long* keys, unsigned n, const Slot* t, unsigned mask,
                         unsigned* rep) {
  const unsigned i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const unsigned long long m = mix64(keys[i]);
  unsigned s = (unsigned)m & mask;
  while (t[s].key != m) s = (s + 1) & mask;
  rep[i] = t[s].min;
}

int main(int argc, char** argv) {
  const unsigned n = argc > 1 ? (unsigned)atoi(argv[1]) : 1310720u;
  const int lg = argc > 2 ? atoi(argv[2]) : 22;  // table slots = 2^lg
  const unsigned S = 1u << lg, mask = S - 1;
  std::vector<unsigned long long> h(n);
  unsigned long long z = 12345;
  const unsigned uniq = n * 7 / 10;
  for (unsigned i = 0; i < n; ++i) {
    z += 0x9E3779B97F4A7C15ull;
    unsigned long long x = z;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    x ^= x >> 31;
    h[i] = i < uniq ? x : h[x % uniq];  // 30 % duplicates of earlier keys
  }
  unsigned long long *keys, *objects;
  Slot* t;
  unsigned* rep;
  CHECK(hipMalloc(&keys, n * 8ull));
  CHECK(hipMalloc(&rep, n * 4ull));
  CHECK(hipMalloc(&t, (size_t)S * sizeof(Slot)));
  CHECK(hipMalloc(&objects, 8));
  CHECK(hipMemcpy(keys, h.data(), n * 8ull, hipMemcpyHostToDevice));
  hipEvent_t e0, e1, e2, e3;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  CHECK(hipEventCreate(&e2));
  CHECK(hipEventCreate(&e3));
  const unsigned blocks = (n + 255) / 256;
  for (int rep_i = 0; rep_i < 8; ++rep_i) {
    CHECK(hipEventRecord(e0));
    CHECK(hipMemsetAsync(t, 0, (size_t)S * sizeof(Slot)));
    CHECK(hipMemsetAsync(objects, 0, 8));
    CHECK(hipEventRecord(e1));
    k_insert<<<blocks, 256>>>(keys, n, t, mask, objects);
    CHECK(hipEventRecord(e2));
    k_lookup<<<blocks, 256>>>(keys, n, t, mask, rep);
    CHECK(hipEventRecord(e3));
    CHECK(hipEventSynchronize(e3));
    float a, b, c;
    CHECK(hipEventElapsedTime(&a, e0, e1));
    CHECK(hipEventElapsedTime(&b, e1, e2));
    CHECK(hipEventElapsedTime(&c, e2, e3));
    unsigned long long obj;
    CHECK(hipMemcpy(&obj, objects, 8, hipMemcpyDeviceToHost));
    printf("{\"n\": %u, \"slots\": %u, \"clear_ms\": %.4f, \"insert_ms\": %.4f, \"lookup_ms\": %.4f, "
           "\"total_ms\": %.4f, \"objects\": %llu}\n", n, S, a, b, c, a + b + c, obj);
  }
  // note: min starts at 0 after the memset in this ubench (timing only); the product
  // would clear mins to 0xFFFFFFFF
  return 0;
}
