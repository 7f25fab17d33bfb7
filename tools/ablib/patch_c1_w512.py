# config-1 pipeline: 512-file gather windows (was 2,048)
s=open('sd_hip_cas.cpp').read()
a="  constexpr size_t GATHER_WINDOW = 2048;"
assert a in s; s=s.replace(a,"  constexpr size_t GATHER_WINDOW = 512;")
open('sd_hip_cas.cpp','w').write(s)
