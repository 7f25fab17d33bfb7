// sd_debug.h — device-side conservation checks of the multi-round LDS kernels (DESIGN.md
// §3b), compiled in only with -DSD_CAS_DEBUG_INVARIANTS=1 (the `debug` target of the
// Makefile: libsd_hip_cas_debug.so).  A violated invariant prints one line from the device
// and counts itself in a per-translation-unit device counter; sd_cas_debug_violations()
// (debug library only, not part of the ABI header) sums the counters, and the GPU test
// suite run against the debug library (tools/gpu_r6_final.sh <tag> suite) fails the test after which
// any counter moved.  Counting instead of trapping keeps a violation from faulting the GPU.
#ifndef SD_DEBUG_H
#define SD_DEBUG_H

#include <hip/hip_runtime.h>
#include <stdint.h>

#if defined(SD_CAS_DEBUG_INVARIANTS) && SD_CAS_DEBUG_INVARIANTS
#define SD_DBG 1
static __device__ unsigned int sd_dbg_violations;
#define SD_DBG_CHECK(cond, fmt, ...)                                                   \
  do {                                                                                 \
    if (!(cond)) {                                                                     \
      atomicAdd(&sd_dbg_violations, 1u);                                               \
      printf("SD_CAS invariant violated (%s:%d): " fmt "\n", __FILE__, __LINE__,      \
             __VA_ARGS__);                                                             \
    }                                                                                  \
  } while (0)
// host accessor of this translation unit's counter
#define SD_DBG_ACCESSOR(name)                                                          \
  uint32_t name() {                                                                    \
    uint32_t v = 0;                                                                    \
    if (hipMemcpyFromSymbol(&v, HIP_SYMBOL(sd_dbg_violations), sizeof v) != hipSuccess) \
      return 0xFFFFFFFFu;                                                              \
    return v;                                                                          \
  }
#else
#define SD_DBG 0
#define SD_DBG_CHECK(cond, fmt, ...) \
  do {                               \
  } while (0)
#define SD_DBG_ACCESSOR(name)
#endif

#endif  // SD_DEBUG_H
