#!/bin/bash
# K2 A/B: ab/k2/*.so vs the in-tree build (tools/prof_packed.py, interleaved twice), then
# the packed-path parity tests on the in-tree build.
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/k2ab
mkdir -p $OUT
cd $R
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread -k "packed or mixed or paths or identifier" > $OUT/pytest.log 2>&1 || { echo PYTEST_FAIL; exit 1; }
for round in 1 2; do
  for lib in $R/ab/k2/libsd_hip_cas_*.so current; do
    name=$(basename $lib .so)
    if [ $lib = current ]; then unset SD_HIP_CAS_LIB; else export SD_HIP_CAS_LIB=$lib; fi
    echo "== $name r$round" >> $OUT/ab.log
    timeout -k 10 300 python3 -u tools/prof_packed.py >> $OUT/ab.log 2>&1 || { echo "TIME_FAIL $name"; exit 1; }
  done
done
echo K2AB_OK
