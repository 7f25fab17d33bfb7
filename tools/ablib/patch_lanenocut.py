# validator lane path without the tail cut (every lane-class buffer one per lane)
s = open('checksum.hip').read()
s = s.replace('#include "blake3_device.hpp"', '#define LANE_TAIL 100000000\n#include "blake3_device.hpp"', 1)
open('checksum.hip', 'w').write(s)
