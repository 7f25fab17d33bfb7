# validator lane kernel in 512-lane workgroups: 96 KiB of stack per workgroup, 1 per CU =
# 2 waves per SIMD without padding
s = open('checksum.hip').read()
a = 'constexpr int LANE_BLOCK = 256;'
assert a in s
s = s.replace(a, 'constexpr int LANE_BLOCK = 512;')
open('checksum.hip', 'w').write(s)
