#!/bin/bash
# A/B timing of K1 builds: every ab/libsd_hip_cas_*.so, then the current in-tree build
# (interleaved twice to expose drift), then the GPU parity suite on the current build.
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/ab
mkdir -p $OUT
cd $R
for round in 1 2; do
  for lib in $R/ab/libsd_hip_cas_*.so current; do
    name=$(basename $lib .so)
    if [ $lib = current ]; then unset SD_HIP_CAS_LIB; else export SD_HIP_CAS_LIB=$lib; fi
    timeout -k 10 300 python3 -u tools/prof_sampled.py --iters 4 > $OUT/time_${name}_r$round.log 2>&1 || { echo "TIME_FAIL $name"; exit 1; }
  done
done
unset SD_HIP_CAS_LIB
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; exit 1; }
echo AB_OK
