# validator lane kernel at 2 waves per SIMD (32 KiB of unused dynamic LDS per workgroup)
s = open('checksum.hip').read()
a = 'sd_b3_batch_lane<<<(uint32_t)((n + LANE_BLOCK - 1) / LANE_BLOCK), LANE_BLOCK, 0, s>>>'
assert a in s
s = s.replace(a, 'sd_b3_batch_lane<<<(uint32_t)((n + LANE_BLOCK - 1) / LANE_BLOCK), LANE_BLOCK, 32768, s>>>')
open('checksum.hip', 'w').write(s)
