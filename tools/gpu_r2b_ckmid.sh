#!/bin/bash
# Validator mid path (65-256 chunk buffers one per wave): checksum tests + shapes.
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r2b_ckmid}
mkdir -p $OUT
cd $R
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -k "checksum" > $OUT/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 300 python3 -u tools/prof_checksums.py > $OUT/validator.log 2>&1 || { echo CK_FAIL; tail -20 $OUT/validator.log; exit 1; }
cut -c1-130 $OUT/validator.log
