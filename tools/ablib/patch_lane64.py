# validator lane path for buffers of <= 64 chunks (5-deep LDS stack, 4 waves/SIMD)
s = open('checksum.hip').read()
s = s.replace('#include "blake3_device.hpp"', '#define LANE_MAX_CHUNKS 64\n#include "blake3_device.hpp"', 1)
open('checksum.hip', 'w').write(s)
