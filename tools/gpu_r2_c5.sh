#!/bin/bash
# Config-5 evidence: the validator tests at multi-GiB sizes, then bench_configs --config 5.
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-c5}
mkdir -p $OUT
cd $R
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -k "checksum" > $OUT/pytest_checksum.log 2>&1 || { echo PYTEST_FAIL; tail -30 $OUT/pytest_checksum.log; exit 1; }
timeout -k 10 600 python3 -u tools/bench_configs.py --config 5 > $OUT/configs5.log 2>&1 || { echo C5_FAIL; tail -20 $OUT/configs5.log; exit 1; }
cat $OUT/configs5.log | grep config
echo C5_OK
