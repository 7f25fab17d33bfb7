# validator lane path for buffers of <= 128 chunks (6-deep LDS stack, 3 waves/SIMD)
s = open('checksum.hip').read()
s = s.replace('#include "blake3_device.hpp"', '#define LANE_MAX_CHUNKS 128\n#include "blake3_device.hpp"', 1)
open('checksum.hip', 'w').write(s)
