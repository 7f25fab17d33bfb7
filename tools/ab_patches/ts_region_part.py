# Instrumentation (timing only): per-block timestamps of sd_region_partition (s_memrealtime,
# 100 MHz, thread 0 after a full wait): entry, keys loaded, histogram + prefill, reservations +
# scan, LDS staging, stores drained; read back with sd_dbg_rpart_ts (tools/ts_region_part.py).
s = open("group_hash.hip").read()
# only sd_region_partition (the big-batch partition below it repeats some of its lines)
CUT = 'extern "C" __global__ void __launch_bounds__(RBIG_THREADS)\nsd_region_partition_big('
s, rest = s.split(CUT, 1)
rest = CUT + rest
def rep(a, b):
    global s
    assert s.count(a) == 1, a
    s = s.replace(a, b)
rep("""extern "C" __global__ void __launch_bounds__(RPART_THREADS)
sd_region_partition(""", """__device__ unsigned long long sd_rpart_ts[4096 * 8];
#define RTS(i) do { if (threadIdx.x == 0) { asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory"); \\
  sd_rpart_ts[(uint64_t)blockIdx.x * 8 + (i)] = wall_clock64(); } } while (0)
extern "C" __global__ void __launch_bounds__(RPART_THREADS)
sd_region_partition(""")
rep("""  const uint32_t tile_n = n - b0 < RPART_TILE ? (uint32_t)(n - b0) : RPART_TILE;
  uint64_t k[RPART_ITEMS];""", """  const uint32_t tile_n = n - b0 < RPART_TILE ? (uint32_t)(n - b0) : RPART_TILE;
  RTS(0);
  uint64_t k[RPART_ITEMS];""")
rep("""  for (uint32_t i = threadIdx.x; i < REGIONS; i += RPART_THREADS) tcnt[i] = 0;
  if (blockIdx.x == 0 && threadIdx.x == 0) { *objects = 0; *spill = 0; }""", """  RTS(1);
  for (uint32_t i = threadIdx.x; i < REGIONS; i += RPART_THREADS) tcnt[i] = 0;
  if (blockIdx.x == 0 && threadIdx.x == 0) { *objects = 0; *spill = 0; }""")
rep("""  // one reservation per non-empty region, then the tile counting-sorted by region in LDS so""",
"""  RTS(2);
  // one reservation per non-empty region, then the tile counting-sorted by region in LDS so""")
rep("""  lds_exclusive_scan(tcnt, tstart, REGIONS);  // (its barriers also publish gbase)
""", """  lds_exclusive_scan(tcnt, tstart, REGIONS);  // (its barriers also publish gbase)
  RTS(3);
""")
rep("""      const uint64_t o = (uint64_t)gbase[b] + (t - tstart[b]);
      if (o < cap) {  // rows past the capacity only counted (the table regroups the region)
        rkeys[(uint64_t)b * cap + o] = kk;
        rfile[(uint64_t)b * cap + o] = sfile[t];
      }
    }
  }
}""", """      const uint64_t o = (uint64_t)gbase[b] + (t - tstart[b]);
      if (o < cap) {  // rows past the capacity only counted (the table regroups the region)
        rkeys[(uint64_t)b * cap + o] = kk;
        rfile[(uint64_t)b * cap + o] = sfile[t];
      }
    }
  }
  RTS(5);
}""")
rep("""      sfile[slot] = (uint32_t)(b0 + t);
    }
  }
  __syncthreads();""", """      sfile[slot] = (uint32_t)(b0 + t);
    }
  }
  __syncthreads();
  RTS(4);""")
s += rest
s += """
extern "C" int sd_dbg_rpart_ts(void* host, size_t bytes) {
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(sdcas::sd_rpart_ts), bytes, 0, hipMemcpyDeviceToHost);
}
"""
open("group_hash.hip", "w").write(s)
