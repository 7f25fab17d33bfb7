#!/bin/bash
# from_paths checks: the path-gather parity tests, then config 1 (10k tmpfs files).
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/paths
mkdir -p $OUT
cd $R
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -p no:cacheprovider --timeout 200 --timeout-method thread -k "paths or identifier or windowed" > $OUT/pytest.log 2>&1 || { echo PYTEST_FAIL; exit 1; }
timeout -k 10 300 python3 -u tools/bench_configs.py --config 1 > $OUT/c1a.log 2>&1 || { echo C1_FAIL; exit 1; }
timeout -k 10 300 python3 -u tools/bench_configs.py --config 1 > $OUT/c1b.log 2>&1 || { echo C1_FAIL; exit 1; }
echo PATHS_OK
