#!/bin/bash
# Build A/B variants of libsd_hip_cas.so that differ only in K3's chunks per lane
# (checksum.hip -DK3_LANE_CHUNKS=N) into ab/; the in-tree build keeps the default.
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
C=$R/spacedrive_amd/csrc
make -C $C -s -j8
mkdir -p $R/ab/k3
for lc in "$@"; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -I$C -I$R/include \
    -DK3_LANE_CHUNKS=$lc -c $C/checksum.hip -o $R/ab/k3/checksum_lc$lc.o
  objs=$(ls $C/build/*.o | grep -v checksum.hip.o)
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $R/ab/k3/libsd_hip_cas_k3lc$lc.so $objs $R/ab/k3/checksum_lc$lc.o
done
