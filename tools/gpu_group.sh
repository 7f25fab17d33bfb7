#!/bin/bash
# GPU pass for the grouping kernels: parity tests of grouping, then timings + kernel stats.
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/grp
mkdir -p $OUT
cd $R
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread -p no:cacheprovider -k "group or partition or shard or multi" > $OUT/pytest.log 2>&1 || { echo PYTEST_FAIL; exit 1; }
timeout -k 10 200 python3 -u tools/bench_group.py > $OUT/bench_group.log 2>&1 || { echo BENCH_FAIL; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/prof -o grp --output-format csv -- python3 $R/tools/bench_group.py > $OUT/prof.log 2>&1 || { echo PROF_FAIL; exit 1; }
echo GROUP_OK
