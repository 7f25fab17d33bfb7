# LDS table insert: CAS first (one LDS round trip per probe) instead of read-then-CAS
s=open('group_hash.hip').read()
a="""    uint64_t cur = tk[slot];
    if (cur == empty) {
      const uint64_t old = atomicCAS((unsigned long long*)&tk[slot], (unsigned long long)empty,
                                     (unsigned long long)k);
      if (old == empty) { ++fresh; cur = k; } else { cur = old; }
    }
    if (cur == k) {
      atomicMin(&tv[slot], v);
      return true;
    }"""
assert a in s
s=s.replace(a,"""    uint64_t cur = atomicCAS((unsigned long long*)&tk[slot], (unsigned long long)empty,
                             (unsigned long long)k);
    if (cur == empty) { ++fresh; cur = k; }
    if (cur == k) {
      atomicMin(&tv[slot], v);
      return true;
    }""",1)
open('group_hash.hip','w').write(s)
