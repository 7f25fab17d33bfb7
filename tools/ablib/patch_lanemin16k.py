# validator lane path from 16,384 buffers up (crossover search)
s = open('checksum.hip').read()
s = s.replace('#include "blake3_device.hpp"', '#define LANE_MIN_BUFFERS 16384\n#include "blake3_device.hpp"', 1)
open('checksum.hip', 'w').write(s)
