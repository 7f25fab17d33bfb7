# K1 at 2 waves per SIMD: 16 KiB of unused dynamic LDS on the 512-lane launch (96 KiB per
# workgroup, one per CU)
s = open('cas_hash.hip').read()
a = 'sd_cas_sampled_kernel<<<(uint32_t)blocks, SAMPLED_BLOCK, 0, s>>>'
assert a in s
s = s.replace(a, 'sd_cas_sampled_kernel<<<(uint32_t)blocks, SAMPLED_BLOCK, 16384, s>>>')
open('cas_hash.hip', 'w').write(s)
