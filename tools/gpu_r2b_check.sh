#!/bin/bash
# Session check on the restored tree: GPU parity suite, smoke, headline bench.
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r2b_check}
mkdir -p $OUT
cd $R
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo SMOKE_FAIL; exit 1; }
timeout -k 10 400 python3 -u bench.py > $OUT/bench.log 2>&1 || { echo BENCH_FAIL; tail -20 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log | cut -c1-600
echo CHECK_OK
