#!/bin/bash
# Batched validator: the new checksum tests + the existing checksum tests.
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r2b_ck}
mkdir -p $OUT
cd $R
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -k "checksum" > $OUT/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -3 $OUT/pytest_gpu.log
