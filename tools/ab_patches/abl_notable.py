# timing-only ablation: one-trip buckets skip the LDS table (no claim, no minimum, no lookup;
# the lookup stores only where an impossible value is read) — what remains is the bounds and
# key loads, the table initialisation, the barriers and the Object atomic
s = open("group_hash.hip").read()
a = """#pragma unroll
      for (int j = 0; j < NI; ++j)
        if (k[j] != empty)
          sl[j] = lds_claim<TBL, SD_ONE_TRIP_READ_FIRST>(tk, home_slot<TBL>(k[j]), k[j], empty, fresh);
#pragma unroll
      for (int j = 0; j < NI; ++j) {
        if (k[j] != empty && sl[j] < TBL) atomicMin(&tv[sl[j]], v[j]);
        ok &= k[j] == empty || sl[j] < TBL;
      }"""
assert s.count(a) == 1
s = s.replace(a, """#pragma unroll
      for (int j = 0; j < NI; ++j) sl[j] = home_slot<TBL>(k[j]);""")
a = """          const uint32_t mv =
              tv[KEEP_SLOT ? sl[j] : lds_find<TBL>(tk, home_slot<TBL>(k[j]), k[j])];
          if (mv != v[j]) out[p[j]] = mv;  // out[] was prefilled with the own value"""
assert s.count(a) == 1
s = s.replace(a, """          const uint32_t mv = tv[sl[j]];
          if (mv == 0x12345u) out[p[j]] = mv;""")
open("group_hash.hip", "w").write(s)
