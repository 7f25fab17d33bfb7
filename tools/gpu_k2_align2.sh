#!/bin/bash
# After switching packed layouts to 128-B alignment: full GPU parity suite, the packing
# A/B timing, and configs 1 (host packing path) and 2 (K2).  Stops at the first failure.
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/k2align2
mkdir -p $OUT
cd $R
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; exit 1; }
for r in 1 2; do
  timeout -k 10 300 python3 -u tools/prof_packed.py >> $OUT/ab.log 2>&1 || { echo TIME_FAIL; exit 1; }
done
timeout -k 10 600 python3 -u tools/bench_configs.py --config 2 --config 1 > $OUT/configs.log 2>&1 || { echo CONFIGS_FAIL; exit 1; }
echo K2ALIGN2_OK
