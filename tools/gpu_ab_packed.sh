#!/bin/bash
# Interleaved K2 timings of A/B builds: gpu_ab_packed.sh <tag> <lib names in tools/ablib>...
# ("cur" = the in-tree build), then the packed parity tests on the in-tree build.
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=$1; shift
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
for i in 1 2 3; do
  for L in "$@"; do
    if [ "$L" = cur ]; then LIB=""; else LIB=$R/tools/ablib/$L.so; fi
    SD_HIP_CAS_LIB=$LIB timeout -k 10 120 python3 tools/ab_packed.py > $OUT/${L}_$i.log 2>&1 || { echo "FAIL $L"; cat $OUT/${L}_$i.log; exit 1; }
    echo "$L $(grep '^{' $OUT/${L}_$i.log)"
  done
done
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "packed or random_cases or layout or whole or config2 or edges" > $OUT/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -30 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
echo AB_OK
