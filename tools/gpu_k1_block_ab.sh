#!/bin/bash
# K1 workgroup-size A/B: sampled-path parity tests on each ab/k1/*.so, then the headline
# bench (no CPU leg) on each variant and the in-tree build, interleaved twice.
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/k1blk
mkdir -p $OUT
cd $R
for lib in $R/ab/k1/libsd_hip_cas_*.so; do
  SD_HIP_CAS_LIB=$lib timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 250 --timeout-method thread -k "sampled or random or quantum" >> $OUT/pytest.log 2>&1 || { echo PYTEST_FAIL; exit 1; }
done
for round in 1 2; do
  for lib in $R/ab/k1/libsd_hip_cas_*.so current; do
    name=$(basename $lib .so)
    if [ $lib = current ]; then unset SD_HIP_CAS_LIB; else export SD_HIP_CAS_LIB=$lib; fi
    echo "== $name r$round" >> $OUT/ab.log
    timeout -k 10 300 python3 -u bench.py --steps 10 --no-cpu-baseline >> $OUT/ab.log 2>&1 || { echo "BENCH_FAIL $name"; exit 1; }
  done
done
echo K1BLK_OK
