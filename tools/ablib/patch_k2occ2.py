# K2 at 2 waves per SIMD: 40 KiB of unused dynamic LDS (80 KiB per workgroup, two per CU)
s = open('cas_hash.hip').read()
a = 'sd_cas_packed_kernel<<<(uint32_t)blocks, 256, 0, s>>>'
assert a in s
s = s.replace(a, 'sd_cas_packed_kernel<<<(uint32_t)blocks, 256, 40960, s>>>')
open('cas_hash.hip', 'w').write(s)
