# K1 at 3 waves per SIMD: always the 256-lane kernel (40 KiB) + 13 KiB of unused dynamic
# LDS = 53 KiB per workgroup, three per CU
s = open('cas_hash.hip').read()
a = 'if (cus && (blocks < cus || (quanta & 1))) {'
assert a in s
s = s.replace(a, 'if (true) {')
a = 'sd_cas_sampled_kernel_256<<<(uint32_t)nb, SAMPLED_BLOCK_NARROW, 0, s>>>'
assert a in s
s = s.replace(a, 'sd_cas_sampled_kernel_256<<<(uint32_t)nb, SAMPLED_BLOCK_NARROW, 13312, s>>>')
open('cas_hash.hip', 'w').write(s)
