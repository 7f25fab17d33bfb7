#!/bin/bash
# Grouping A/B: the variant's grouping parity tests, then tools/bench_group.py on
# ab/grp/*.so and the in-tree build, interleaved twice.  Stops at the first failure.
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/grpab2
mkdir -p $OUT
cd $R
for lib in $R/ab/grp/libsd_hip_cas_*.so; do
  SD_HIP_CAS_LIB=$lib timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 250 --timeout-method thread -k "group or shard or multi or bench_scale or headline" >> $OUT/pytest.log 2>&1 || { echo PYTEST_FAIL; exit 1; }
done
for round in 1 2; do
  for lib in $R/ab/grp/libsd_hip_cas_*.so current; do
    name=$(basename $lib .so)
    if [ $lib = current ]; then unset SD_HIP_CAS_LIB; else export SD_HIP_CAS_LIB=$lib; fi
    echo "== $name r$round" >> $OUT/ab.log
    timeout -k 10 300 python3 -u tools/bench_group.py >> $OUT/ab.log 2>&1 || { echo "GROUP_FAIL $name"; exit 1; }
  done
done
echo GRPAB2_OK
