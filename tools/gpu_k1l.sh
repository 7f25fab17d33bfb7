#!/bin/bash
# GPU parity suite (all kernel shapes) then the K1L / K1 crossover sweep.
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/k1l
mkdir -p $OUT
cd $R
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; exit 1; }
timeout -k 10 300 python3 -u tools/latency_sweep.py > $OUT/sweep.log 2>&1 || { echo SWEEP_FAIL; exit 1; }
echo K1L_OK
