# small batches: two gather windows (the second gathered while the first is copied + hashed)
s=open('sd_hip_cas.cpp').read()
a="  constexpr size_t GATHER_WINDOW = 2048;"
assert a in s
s=s.replace(a,"  const size_t GATHER_WINDOW = n <= 4096 ? std::max<size_t>(32, (n + 1) / 2) : 2048;")
open('sd_hip_cas.cpp','w').write(s)
