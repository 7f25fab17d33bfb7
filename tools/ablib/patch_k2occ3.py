# K2 at 3 waves per SIMD: 8 KiB of unused dynamic LDS (48 KiB per workgroup, three per CU)
s = open('cas_hash.hip').read()
a = 'sd_cas_packed_kernel<<<(uint32_t)blocks, 256, 0, s>>>'
assert a in s
s = s.replace(a, 'sd_cas_packed_kernel<<<(uint32_t)blocks, 256, 8192, s>>>')
open('cas_hash.hip', 'w').write(s)
