# diagnosis: bucket_min without inserts and stores (loads + table init only)
s=open('group_hash.hip').read()
a="          if (mv != v[j]) out[p[j]] = mv;  // out[] was prefilled with the own value"
assert a in s; s=s.replace(a,"          if (mv == 0xFFFFFFFEu) out[p[j]] = mv;")
a="      if (k[j] != empty) ok &= lds_insert<TBL>(tk, tv, sl[j], k[j], v[j], empty, fresh);"
assert a in s; s=s.replace(a,"      if (k[j] == 0x123456789ull) ok &= lds_insert<TBL>(tk, tv, sl[j], k[j], v[j], empty, fresh);")
open('group_hash.hip','w').write(s)
