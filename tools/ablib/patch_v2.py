s=open('group_hash.hip').read()
a="""          const uint32_t mv = tv[sl[j]];"""
b="""          const uint32_t mv = tv[lds_find<TBL>(tk, (uint32_t)k[j] & (TBL - 1), k[j])];"""
assert a in s; s=s.replace(a,b); open('group_hash.hip','w').write(s)
