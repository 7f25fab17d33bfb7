// ubench_bucketload.hip — the memory side of the fine bucket tables (sd_bucket_min) alone:
// 8,192 buckets of ~1,526 rows (12.5 M rows of u64 key + u32 pos, bucket-contiguous), each
// read by 512 lanes x 4 rows, reduced to one value per bucket (no LDS table).
//   A: one workgroup per bucket (the kernel's grid);
//   B: a resident grid (3 workgroups per CU) walking the buckets, no prefetch;
//   C: B with the next bucket's rows loaded (raw, no use) while the current one is reduced;
//   A/C after W: the same right after a kernel that rewrote every row (the refine's output
//   is read by the tables straight after it is written).
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/ubench_bucketload tools/ubench_bucketload.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include <vector>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

constexpr int T = 512, NI = 4;

__device__ __forceinline__ uint64_t reduce_rows(const uint64_t* __restrict__ k, const uint32_t* __restrict__ p,
                                                uint64_t s, uint64_t e) {
  uint64_t acc = 0;
#pragma unroll
  for (int j = 0; j < NI; ++j) {
    const uint64_t i = s + (uint64_t)j * T + threadIdx.x;
    const uint64_t c = i < e ? i : e - 1;
    const uint64_t kk = k[c];
    const uint32_t pp = p[c];
    acc += i < e ? (kk ^ pp) : 0;
  }
  return acc;
}

__global__ void __launch_bounds__(T) per_bucket(const uint64_t* __restrict__ k, const uint32_t* __restrict__ p,
                                                const uint32_t* __restrict__ starts, uint32_t nb, uint64_t n,
                                                uint64_t* __restrict__ out) {
  __shared__ uint64_t pad[6144];  // the tables' LDS footprint: 3 workgroups per CU
  const uint32_t b = blockIdx.x;
  const uint64_t s = starts[b], e = b + 1 < nb ? starts[b + 1] : n;
  uint64_t acc = reduce_rows(k, p, s, e);
  pad[threadIdx.x] = acc;
  __syncthreads();
  if (threadIdx.x == 0) out[b] = pad[0] + pad[T - 1];
}

// A plus the tables' Object count: one device-scope atomic add per workgroup on ONE counter
// (objects != nullptr) or on one of 64 counters, each on its own 128-B line (shards)
__global__ void __launch_bounds__(T) per_bucket_atomic(const uint64_t* __restrict__ k, const uint32_t* __restrict__ p,
                                                       const uint32_t* __restrict__ starts, uint32_t nb, uint64_t n,
                                                       uint64_t* __restrict__ out, unsigned long long* __restrict__ objects,
                                                       uint32_t shards) {
  __shared__ uint64_t pad[6144];
  const uint32_t b = blockIdx.x;
  const uint64_t s = starts[b], e = b + 1 < nb ? starts[b + 1] : n;
  uint64_t acc = reduce_rows(k, p, s, e);
  pad[threadIdx.x] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    out[b] = pad[0] + pad[T - 1];
    atomicAdd(objects + (b % shards) * 16, (unsigned long long)(e - s));
  }
}

__global__ void __launch_bounds__(T) resident(const uint64_t* __restrict__ k, const uint32_t* __restrict__ p,
                                              const uint32_t* __restrict__ starts, uint32_t nb, uint64_t n,
                                              uint64_t* __restrict__ out) {
  __shared__ uint64_t pad[6144];
  for (uint32_t b = blockIdx.x; b < nb; b += gridDim.x) {
    const uint64_t s = starts[b], e = b + 1 < nb ? starts[b + 1] : n;
    uint64_t acc = reduce_rows(k, p, s, e);
    pad[threadIdx.x] = acc;
    __syncthreads();
    if (threadIdx.x == 0) out[b] = pad[0] + pad[T - 1];
    __syncthreads();
  }
}

__global__ void __launch_bounds__(T) resident_prefetch(const uint64_t* __restrict__ k, const uint32_t* __restrict__ p,
                                                       const uint32_t* __restrict__ starts, uint32_t nb, uint64_t n,
                                                       uint64_t* __restrict__ out) {
  __shared__ uint64_t pad[6144];
  const uint32_t G = gridDim.x;
  uint32_t b = blockIdx.x;
  if (b >= nb) return;
  uint64_t s = starts[b], e = b + 1 < nb ? starts[b + 1] : n;
  uint64_t ka[NI], kb[NI];
  uint32_t pa[NI], pb[NI];
  auto load = [&](uint64_t s0, uint64_t e0, uint64_t (&kk)[NI], uint32_t (&pp)[NI]) {
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      const uint64_t i = s0 + (uint64_t)j * T + threadIdx.x;
      const uint64_t c = i < e0 ? i : (e0 ? e0 - 1 : 0);
      kk[j] = k[c];
      pp[j] = p[c];
    }
  };
  load(s, e, ka, pa);
  auto step = [&](uint64_t (&kc)[NI], uint32_t (&pc)[NI], uint64_t (&kx)[NI], uint32_t (&px)[NI]) {
    const uint32_t bn = b + G;
    const uint64_t s1 = bn < nb ? starts[bn] : 0, e1 = bn < nb ? (bn + 1 < nb ? starts[bn + 1] : n) : 0;
    load(s1, e1, kx, px);  // in flight while bucket b is reduced
    uint64_t acc = 0;
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      const uint64_t i = s + (uint64_t)j * T + threadIdx.x;
      acc += i < e ? (kc[j] ^ pc[j]) : 0;
    }
    pad[threadIdx.x] = acc;
    __syncthreads();
    if (threadIdx.x == 0) out[b] = pad[0] + pad[T - 1];
    __syncthreads();
    b = bn; s = s1; e = e1;
    return b < nb;
  };
  while (step(ka, pa, kb, pb) && step(kb, pb, ka, pa)) {
  }
}

__global__ void rewrite(uint64_t* __restrict__ k, uint32_t* __restrict__ p, uint64_t n, uint32_t salt) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    k[i] = i * 0x9E3779B97F4A7C15ull + salt;
    p[i] = (uint32_t)i ^ salt;
  }
}

int main() {
  const uint64_t n = 12500000;
  const uint32_t nb = 8192;
  std::vector<uint32_t> st(nb);
  for (uint32_t b = 0; b < nb; ++b) st[b] = (uint32_t)(n * b / nb);
  uint64_t *k, *out;
  uint32_t *p, *starts;
  CHECK(hipMalloc(&k, n * 8));
  CHECK(hipMalloc(&p, n * 4));
  CHECK(hipMalloc(&starts, nb * 4));
  CHECK(hipMalloc(&out, nb * 8));
  CHECK(hipMemset(k, 1, n * 8));
  CHECK(hipMemset(p, 2, n * 4));
  CHECK(hipMemcpy(starts, st.data(), nb * 4, hipMemcpyHostToDevice));
  int per_cu = 0, cus = 0;
  CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, reinterpret_cast<const void*>(resident), T, 0));
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const uint32_t grid = per_cu * cus;
  hipEvent_t a, bq;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&bq));
  auto timeit = [&](const char* name, auto launch) -> int {
    for (int w = 0; w < 3; ++w) launch();
    CHECK(hipDeviceSynchronize());
    float best = 1e9f, sum = 0;
    for (int r = 0; r < 10; ++r) {
      CHECK(hipEventRecord(a, 0));
      launch();
      CHECK(hipEventRecord(bq, 0));
      CHECK(hipEventSynchronize(bq));
      float ms = 0;
      CHECK(hipEventElapsedTime(&ms, a, bq));
      best = ms < best ? ms : best;
      sum += ms;
    }
    printf("%-22s best %7.1f us  mean %7.1f us  (%5.2f TB/s of 12 B/row)\n", name, best * 1e3, sum / 10 * 1e3,
           12.0 * n / (best * 1e-3) / 1e12);
    return 0;
  };
  printf("resident grid %u (%d per CU x %d CUs)\n", grid, per_cu, cus);
  if (timeit("A one WG per bucket", [&] { per_bucket<<<nb, T>>>(k, p, starts, nb, n, out); })) return 1;
  if (timeit("B resident", [&] { resident<<<grid, T>>>(k, p, starts, nb, n, out); })) return 1;
  if (timeit("C resident+prefetch", [&] { resident_prefetch<<<grid, T>>>(k, p, starts, nb, n, out); })) return 1;
  // after a rewrite of the rows: time the reader alone (events between the two launches)
  auto after = [&](const char* name, auto launch) -> int {
    float best = 1e9f, wbest = 1e9f;
    for (int r = 0; r < 10; ++r) {
      hipEvent_t w0;
      CHECK(hipEventCreate(&w0));
      CHECK(hipEventRecord(w0, 0));
      rewrite<<<2048, 256>>>(k, p, n, (uint32_t)r);
      CHECK(hipEventRecord(a, 0));
      launch();
      CHECK(hipEventRecord(bq, 0));
      CHECK(hipEventSynchronize(bq));
      float ms = 0, wms = 0;
      CHECK(hipEventElapsedTime(&ms, a, bq));
      CHECK(hipEventElapsedTime(&wms, w0, a));
      best = ms < best ? ms : best;
      wbest = wms < wbest ? wms : wbest;
      CHECK(hipEventDestroy(w0));
    }
    printf("%-22s best %7.1f us  (rewrite before it: %6.1f us)\n", name, best * 1e3, wbest * 1e3);
    return 0;
  };
  unsigned long long* obj;
  CHECK(hipMalloc(&obj, 64 * 128));
  CHECK(hipMemset(obj, 0, 64 * 128));
  if (timeit("A + 1 counter atomic", [&] { per_bucket_atomic<<<nb, T>>>(k, p, starts, nb, n, out, obj, 1); })) return 1;
  if (timeit("A + 64 counter atomics", [&] { per_bucket_atomic<<<nb, T>>>(k, p, starts, nb, n, out, obj, 64); })) return 1;
  if (after("A after rewrite", [&] { per_bucket<<<nb, T>>>(k, p, starts, nb, n, out); })) return 1;
  if (after("C after rewrite", [&] { resident_prefetch<<<grid, T>>>(k, p, starts, nb, n, out); })) return 1;
  return 0;
}
