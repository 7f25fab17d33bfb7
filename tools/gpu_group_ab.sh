#!/bin/bash
# Grouping check: GPU grouping parity tests, then bench (group ms at 1.31M keys) and the
# 12.5M-key grouping sweep.
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/grp
mkdir -p $OUT
cd $R
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 250 --timeout-method thread -k "group or shard or multi or bench_scale" > $OUT/pytest.log 2>&1 || { echo PYTEST_FAIL; exit 1; }
timeout -k 10 300 python3 -u bench.py --steps 5 --no-cpu-baseline > $OUT/bench.log 2>&1 || { echo BENCH_FAIL; exit 1; }
timeout -k 10 300 python3 -u tools/bench_group.py > $OUT/group.log 2>&1 || { echo GROUP_FAIL; exit 1; }
echo GRP_OK
