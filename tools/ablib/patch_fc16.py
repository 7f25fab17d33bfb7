# file_checksum: 16 pool readers per segment (was 8)
s=open('sd_hip_cas.cpp').read()
a="    c->pool.run((unsigned)std::min<uint64_t>(8, npieces), [&]() {"
assert a in s; s=s.replace(a,"    c->pool.run((unsigned)std::min<uint64_t>(16, npieces), [&]() {")
open('sd_hip_cas.cpp','w').write(s)
