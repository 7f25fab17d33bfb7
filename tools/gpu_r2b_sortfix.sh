#!/bin/bash
# Downsweep race fix: the repeated large sort, the grouping/sort tests, then the 100M config-4 test.
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r2b_sortfix}
mkdir -p $OUT
cd $R
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -k "sort_pairs or group or config4 or multi_device" > $OUT/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -3 $OUT/pytest_gpu.log
