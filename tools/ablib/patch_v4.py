# 2,048-slot tables (24 KiB LDS: 4 workgroups/CU) with a 1,024-key bucket target
s=open('group_hash.hip').read()
for a,b in [("constexpr uint32_t TABLE = 4096; ", "constexpr uint32_t TABLE = 2048; "),
            ("constexpr uint64_t TARGET_PER_BUCKET = 1536;", "constexpr uint64_t TARGET_PER_BUCKET = 1024;")]:
    assert a in s; s=s.replace(a,b)
open('group_hash.hip','w').write(s)
