# diagnosis: scatter without its global key/pos stores (timing only)
s=open('group_hash.hip').read()
a="""      const uint32_t dest = gcur[b] + (t - tstart[b]);
      out_keys[dest] = kk;
      out_pos[dest] = spos[t];"""
assert a in s; s=s.replace(a,"""      const uint32_t dest = gcur[b] + (t - tstart[b]);
      if (kk == 0x123456789ull) { out_keys[dest] = kk; out_pos[dest] = spos[t]; }""")
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
