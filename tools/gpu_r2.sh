#!/bin/bash
# Round-2 GPU pass: parity suite (-m gpu), smoke, headline bench.  Usage: gpu_r2.sh <tag> [pytest -k expr]
# Each GPU step has its own time limit; stop at the first failure.
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-r2}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
K=()
if [ -n "$2" ]; then K=(-k "$2"); fi
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread "${K[@]}" > $OUT/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -30 $OUT/pytest_gpu.log; exit 1; }
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo SMOKE_FAIL; exit 1; }
timeout -k 10 400 python3 -u bench.py --steps 20 --warmup 5 > $OUT/bench.log 2>&1 || { echo BENCH_FAIL; tail -20 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log
echo R2_OK
