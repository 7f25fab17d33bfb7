# Instrumentation (timing only): per-block timestamps of sd_part_scatter_mix (s_memrealtime,
# 100 MHz, thread 0 after a full wait): entry, after the totals/scan prologue, after each trip
# (up to 6), read back with sd_dbg_scatter_ts (tools/ts_scatter.py).
s = open("group_hash.hip").read()
def rep(a, b):
    global s
    assert s.count(a) == 1, a
    s = s.replace(a, b)
rep("""template <int MODE, bool STORE_ALL>
__device__ void part_scatter_body(""", """__device__ unsigned long long sd_scatter_ts[4096 * 8];
#define STS(i) do { if (MODE == 0 && threadIdx.x == 0 && (i) < 8) { asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory"); \\
  sd_scatter_ts[(uint64_t)blockIdx.x * 8 + (i)] = wall_clock64(); } } while (0)
template <int MODE, bool STORE_ALL>
__device__ void part_scatter_body(""")
rep("""  const bool staged = nb <= STAGED_MAX_NB;
  const uint32_t mine = blockIdx.x % repl;""", """  const bool staged = nb <= STAGED_MAX_NB;
  STS(0);
  const uint32_t mine = blockIdx.x % repl;""")
rep("""    for (uint32_t b = threadIdx.x; b < nb; b += PART_THREADS) tcnt[b] = 0;
    __syncthreads();
    auto bfn = [nb](uint64_t x) { return bucket_of(x, nb); };""", """    for (uint32_t b = threadIdx.x; b < nb; b += PART_THREADS) tcnt[b] = 0;
    __syncthreads();
    STS(1);
    uint32_t tno = 0;
    auto bfn = [nb](uint64_t x) { return bucket_of(x, nb); };""")
rep("""                        [&]() { load_trip(nbase); });  // in flight during this trip
    }
    return;""", """                        [&]() { load_trip(nbase); });  // in flight during this trip
      ++tno;
      STS(1 + tno);
    }
    return;""")
s += """
extern "C" int sd_dbg_scatter_ts(void* host, size_t bytes) {
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(sdcas::sd_scatter_ts), bytes, 0, hipMemcpyDeviceToHost);
}
"""
open("group_hash.hip", "w").write(s)
