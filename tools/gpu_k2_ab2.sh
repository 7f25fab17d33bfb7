#!/bin/bash
# K2 A/B with the variant's own parity check: packed-path GPU tests on ab/k2/*.so, then
# tools/prof_packed.py interleaved twice against the in-tree build.
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/k2ab2
mkdir -p $OUT
cd $R
for lib in $R/ab/k2/libsd_hip_cas_*.so; do
  SD_HIP_CAS_LIB=$lib timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread -k "packed or mixed or random or identifier" >> $OUT/pytest.log 2>&1 || { echo PYTEST_FAIL; exit 1; }
done
for round in 1 2; do
  for lib in $R/ab/k2/libsd_hip_cas_*.so current; do
    name=$(basename $lib .so)
    if [ $lib = current ]; then unset SD_HIP_CAS_LIB; else export SD_HIP_CAS_LIB=$lib; fi
    echo "== $name r$round" >> $OUT/ab.log
    timeout -k 10 300 python3 -u tools/prof_packed.py >> $OUT/ab.log 2>&1 || { echo "TIME_FAIL $name"; exit 1; }
  done
done
echo K2AB2_OK
