# file_checksum: 16 pool readers per segment and 2 MiB pieces (32 per segment)
s=open('sd_hip_cas.cpp').read()
a="    c->pool.run((unsigned)std::min<uint64_t>(8, npieces), [&]() {"
assert a in s; s=s.replace(a,"    c->pool.run((unsigned)std::min<uint64_t>(16, npieces), [&]() {")
a="  constexpr uint64_t PIECE = 4ull << 20;"
assert a in s; s=s.replace(a,"  constexpr uint64_t PIECE = 2ull << 20;")
open('sd_hip_cas.cpp','w').write(s)
