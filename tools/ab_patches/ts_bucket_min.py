# Instrumentation (timing only): per-workgroup phase timestamps of sd_bucket_min, read back
# with sd_dbg_bucket_ts (tools/ts_bucket_min.py).  s_memrealtime (100 MHz) on thread 0 after
# a full wait, at: entry, bucket bounds loaded, table initialised + keys loaded (first
# barrier), inserts done (post-loop barrier), lookups + stores done.
s = open("group_hash.hip").read()
def rep(a, b):
    global s
    assert s.count(a) == 1, a
    s = s.replace(a, b)
hdr = ("template <uint32_t TBL, int THREADS, int NI, bool KEEP_SLOT>\n" if "int NI, bool KEEP_SLOT>" in s
       else "template <uint32_t TBL, int THREADS, bool KEEP_SLOT>\n") + "__device__ __forceinline__ void bucket_min("
rep(hdr, """__device__ unsigned long long sd_bucket_ts[65536 * 5];
#define TS(i) do { if (threadIdx.x == 0 && TBL == TABLE) { asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory"); \\
  sd_bucket_ts[(uint64_t)bucket * 5 + (i)] = wall_clock64(); } } while (0)
""" + hdr)
rep("""  const uint32_t b = bucket;
  // the chain's bucket totals""", """  const uint32_t b = bucket;
  TS(0);
  // the chain's bucket totals""")
rep("""  if (s == e && !whole) return;  // uniform for the whole workgroup""", """  if (threadIdx.x == 0 && s == 0xFFFFFFFFFFFFull) sd_bucket_ts[0] = e;
  TS(1);
  if (s == e && !whole) return;  // uniform for the whole workgroup""")
rep("""    __syncthreads();  // table initialised (first trip) / the previous trip's flag visible
""", """    __syncthreads();  // table initialised (first trip) / the previous trip's flag visible
    if (trip == 0) TS(2);
""")
rep("""  const bool overflow = whole || (ovf[0] | ovf[1]);""", """  TS(3);
  const bool overflow = whole || (ovf[0] | ovf[1]);""")
rep("""    if (threadIdx.x == 0) atomicAdd(objects, (unsigned long long)distinct);
    return;""", """    TS(4);
    if (threadIdx.x == 0) atomicAdd(objects, (unsigned long long)distinct);
    return;""")
s += """
extern "C" int sd_dbg_bucket_ts(void* host, size_t bytes) {
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(sdcas::sd_bucket_ts), bytes, 0, hipMemcpyDeviceToHost);
}
"""
open("group_hash.hip", "w").write(s)
