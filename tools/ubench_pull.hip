// ubench_pull.hip — host -> HBM transfer of the job step's streamed pieces (128 KiB..4 MiB
// of pinned host memory): SDMA (hipMemcpyAsync) against a shader pull (each lane loads 16-B
// quads of the host buffer over PCIe and stores them to HBM) at several grid shapes, one
// piece at a time on one stream, timed by HIP events (median of 50).  Prices the transfer
// leg of the 100-file job step (profiles/r04_jobstep_*).
// Second table: the same transfers of a piece the CPU has JUST written (as the job step's
// pread gather leaves it: dirty lines in the host caches), written with plain stores, with
// non-temporal stores, or with plain stores + clflushopt.
// Build: hipcc --offload-arch=gfx950 -O3 -mavx2 -mclflushopt -o tools/ubench_pull tools/ubench_pull.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <immintrin.h>

#include <algorithm>
#include <vector>

#define CHECK(x)                                                                  \
  do {                                                                            \
    hipError_t e = (x);                                                           \
    if (e != hipSuccess) {                                                        \
      fprintf(stderr, "%s: %s (%s:%d)\n", #x, hipGetErrorString(e), __FILE__, __LINE__); \
      exit(1);                                                                    \
    }                                                                             \
  } while (0)

// grid-stride over quads, U quads per lane in flight (wave-contiguous per load)
template <int U>
__global__ void __launch_bounds__(256) pull(const uint4* __restrict__ src, uint4* __restrict__ dst,
                                            uint64_t quads) {
  const uint64_t step = (uint64_t)gridDim.x * 256;
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < quads; i += step * U) {
    uint4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (i + u * step < quads) v[u] = src[i + u * step];
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (i + u * step < quads) dst[i + u * step] = v[u];
  }
}

// each workgroup moves one contiguous span (span quads), U quads per lane per trip
template <int U>
__global__ void __launch_bounds__(256) pull_span(const uint4* __restrict__ src, uint4* __restrict__ dst,
                                                 uint64_t quads, uint64_t span) {
  const uint64_t b0 = (uint64_t)blockIdx.x * span;
  const uint64_t e = b0 + span < quads ? b0 + span : quads;
  for (uint64_t i = b0 + threadIdx.x; i < e; i += 256 * U) {
    uint4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (i + u * 256 < e) v[u] = src[i + u * 256];
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (i + u * 256 < e) dst[i + u * 256] = v[u];
  }
}

// 64-lane workgroups: the same bytes over as many CUs as possible
template <int U>
__global__ void __launch_bounds__(64) pull64(const uint4* __restrict__ src, uint4* __restrict__ dst,
                                             uint64_t quads) {
  const uint64_t step = (uint64_t)gridDim.x * 64;
  for (uint64_t i = (uint64_t)blockIdx.x * 64 + threadIdx.x; i < quads; i += step * U) {
    uint4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (i + u * step < quads) v[u] = src[i + u * step];
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (i + u * step < quads) dst[i + u * step] = v[u];
  }
}

typedef void (*launch_fn)(const uint4*, uint4*, uint64_t, hipStream_t);

template <int U>
static void l_stride(const uint4* s, uint4* d, uint64_t q, hipStream_t st) {
  uint64_t blocks = (q + 256 * U - 1) / (256 * U);
  if (blocks > 2048) blocks = 2048;
  pull<U><<<(unsigned)blocks, 256, 0, st>>>(s, d, q);
}
template <int U>
static void l_wave(const uint4* s, uint4* d, uint64_t q, hipStream_t st) {
  uint64_t blocks = (q + 64 * U - 1) / (64 * U);
  if (blocks > 8192) blocks = 8192;
  pull64<U><<<(unsigned)blocks, 64, 0, st>>>(s, d, q);
}
template <int U, int SPANQ>
static void l_span(const uint4* s, uint4* d, uint64_t q, hipStream_t st) {
  const uint64_t blocks = (q + SPANQ - 1) / SPANQ;
  pull_span<U><<<(unsigned)blocks, 256, 0, st>>>(s, d, q, SPANQ);
}

int main() {
  const size_t maxb = 4u << 20;
  void* host[2];
  CHECK(hipHostMalloc(&host[0], maxb, hipHostMallocDefault));
  CHECK(hipHostMalloc(&host[1], maxb, hipHostMallocNonCoherent));
  memset(host[0], 0x5a, maxb);
  memset(host[1], 0xa5, maxb);
  void* dev;
  CHECK(hipMalloc(&dev, maxb));
  hipStream_t st;
  CHECK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  struct V { const char* name; launch_fn f; };
  const V vars[] = {
      {"sdma hipMemcpyAsync", nullptr},
      {"pull stride U1", l_stride<1>},
      {"pull stride U4", l_stride<4>},
      {"pull stride U8", l_stride<8>},
      {"pull span 4KiB U1", l_span<1, 256>},
      {"pull span 16KiB U4", l_span<4, 1024>},
      {"pull span 8KiB U2", l_span<2, 512>},
      {"pull span 32KiB U8", l_span<8, 2048>},
      {"pull wave64 U1", l_wave<1>},
      {"pull wave64 U2", l_wave<2>},
  };
  const size_t sizes[] = {128u << 10, 512u << 10, 1u << 20, 4u << 20};
  for (int h = 0; h < 2; ++h) {
    printf("# host buffer: %s\n", h ? "hipHostMallocNonCoherent" : "hipHostMallocDefault");
    for (size_t sz : sizes) {
      for (const V& v : vars) {
        std::vector<float> ts;
        for (int r = 0; r < 60; ++r) {
          CHECK(hipEventRecord(a, st));
          if (v.f)
            v.f((const uint4*)host[h], (uint4*)dev, sz / 16, st);
          else
            CHECK(hipMemcpyAsync(dev, host[h], sz, hipMemcpyHostToDevice, st));
          CHECK(hipEventRecord(b, st));
          CHECK(hipEventSynchronize(b));
          float ms;
          CHECK(hipEventElapsedTime(&ms, a, b));
          if (r >= 10) ts.push_back(ms);
        }
        std::sort(ts.begin(), ts.end());
        const double med = ts[ts.size() / 2] * 1e3;
        printf("%-22s %5zu KiB  %7.1f us  %6.1f GB/s\n", v.name, sz >> 10, med, sz / (med * 1e3));
      }
    }
  }
  // pieces the CPU has just written
  const char* modes[] = {"plain stores", "nt stores", "stores+clflushopt"};
  const V vars2[] = {
      {"sdma hipMemcpyAsync", nullptr},
      {"pull stride U1", l_stride<1>},
      {"pull stride U4", l_stride<4>},
      {"pull span 8KiB U2", l_span<2, 512>},
      {"pull wave64 U1", l_wave<1>},
  };
  for (int m = 0; m < 3; ++m) {
    printf("# dirty piece (hipHostMallocDefault), CPU wrote it with %s just before\n", modes[m]);
    for (size_t sz : sizes) {
      for (const V& v : vars2) {
        std::vector<float> ts;
        for (int r = 0; r < 60; ++r) {
          unsigned char* hp = (unsigned char*)host[0];
          if (m == 1) {
            const __m256i x = _mm256_set1_epi8((char)r);
            for (size_t o = 0; o < sz; o += 32) _mm256_stream_si256((__m256i*)(hp + o), x);
            _mm_sfence();
          } else {
            memset(hp, r, sz);
            if (m == 2) {
              for (size_t o = 0; o < sz; o += 64) _mm_clflushopt(hp + o);
              _mm_sfence();
            }
          }
          CHECK(hipEventRecord(a, st));
          if (v.f)
            v.f((const uint4*)host[0], (uint4*)dev, sz / 16, st);
          else
            CHECK(hipMemcpyAsync(dev, host[0], sz, hipMemcpyHostToDevice, st));
          CHECK(hipEventRecord(b, st));
          CHECK(hipEventSynchronize(b));
          float ms;
          CHECK(hipEventElapsedTime(&ms, a, b));
          if (r >= 10) ts.push_back(ms);
        }
        std::sort(ts.begin(), ts.end());
        const double med = ts[ts.size() / 2] * 1e3;
        printf("%-22s %5zu KiB  %7.1f us  %6.1f GB/s\n", v.name, sz >> 10, med, sz / (med * 1e3));
      }
    }
  }
  memcpy(host[1], host[0], maxb);
  // verify the last pull
  std::vector<unsigned char> chk(maxb);
  CHECK(hipMemcpy(chk.data(), dev, maxb, hipMemcpyDeviceToHost));
  printf("check: %s\n", memcmp(chk.data(), host[1], maxb) == 0 ? "ok" : "MISMATCH");
  return 0;
}
