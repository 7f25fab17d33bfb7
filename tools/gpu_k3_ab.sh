#!/bin/bash
# K3 chunks-per-lane A/B (ab/k3/*.so vs the in-tree default), interleaved twice, then the
# GPU checksum parity tests on the in-tree build.
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/k3ab
mkdir -p $OUT
cd $R
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider -k checksum > $OUT/pytest_checksum.log 2>&1 || { echo PYTEST_FAIL; exit 1; }
for round in 1 2; do
  for lib in $R/ab/k3/libsd_hip_cas_*.so current; do
    name=$(basename $lib .so)
    if [ $lib = current ]; then unset SD_HIP_CAS_LIB; else export SD_HIP_CAS_LIB=$lib; fi
    timeout -k 10 300 python3 -u tools/prof_checksum.py --gib 64 >> $OUT/k3_ab.log 2>$OUT/err_${name}.log || { echo "TIME_FAIL $name"; exit 1; }
  done
done
echo K3AB_OK
