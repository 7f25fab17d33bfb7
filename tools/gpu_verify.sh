#!/bin/bash
# Quick re-check of a rebuilt tree: parity suite, smoke, headline bench. Stops at the first failure.
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/verify
mkdir -p $OUT
cd $R
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; exit 1; }
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo SMOKE_FAIL; exit 1; }
timeout -k 10 400 python3 -u bench.py > $OUT/bench.log 2>&1 || { echo BENCH_FAIL; exit 1; }
echo VERIFY_OK
