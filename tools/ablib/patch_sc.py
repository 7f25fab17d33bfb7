# diagnosis: scatter = totals sum + scan + key loads only (returns before the trip)
s=open('group_hash.hip').read()
a="""    for (uint64_t base = lo; base < hi; base += PART_TILE) {
      if (base != lo) load_trip(base);"""
assert a in s; s=s.replace(a,"""    if (k[0] == 0x123456789ull && k[3] == 7ull) out_keys[0] = k[1];
    return;
    for (uint64_t base = lo; base < hi; base += PART_TILE) {
      if (base != lo) load_trip(base);""")
open('group_hash.hip','w').write(s)
# (and bucket_min never stores: the partition it reads is garbage in this diagnosis build)
s=open('group_hash.hip').read()
a="          if (mv != v[j]) out[p[j]] = mv;  // out[] was prefilled with the own value"
assert a in s; s=s.replace(a,"          if (mv == 0xFFFFFFFEu && p[j] < n) out[p[j]] = mv;")
a="            if (mv != (vals ? vals[p[j]] : p[j])) out[p[j]] = mv;"
assert a in s; s=s.replace(a,"            if (mv == 0xFFFFFFFEu && p[j] < n) out[p[j]] = mv;")
a="    if (mv != (vals ? vals[pp] : pp)) out[pp] = mv;"
assert a in s; s=s.replace(a,"    if (mv == 0xFFFFFFFEu && pp < n) out[pp] = mv;")
a="    g_insert(gk, gv, cap, (kk & 0xFFFFFFFFull) % cap, kk, vals ? vals[pp] : pp, empty, fresh);"
assert a in s; s=s.replace(a,"    g_insert(gk, gv, cap, (kk & 0xFFFFFFFFull) % cap, kk, pp, empty, fresh);")
open('group_hash.hip','w').write(s)
