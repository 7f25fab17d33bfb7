# diagnosis: bucket_min without the output stores (timing only; results wrong)
s=open('group_hash.hip').read()
a="          if (mv != v[j]) out[p[j]] = mv;  // out[] was prefilled with the own value"
assert a in s; s=s.replace(a,"          if (mv == 0xFFFFFFFEu) out[p[j]] = mv;")
open('group_hash.hip','w').write(s)
