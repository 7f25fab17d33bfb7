#!/bin/bash
# LSD fallback evidence: the tests that run the sort path (forced SORT method, sort_pairs,
# multi-device grouping), then bench_group's LSD timing and a FETCH_SIZE pass on it.
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-lsd}
mkdir -p $OUT
cd $R
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -k "group or sort or multi or headline" > $OUT/pytest_lsd.log 2>&1 || { echo PYTEST_FAIL; tail -40 $OUT/pytest_lsd.log; exit 1; }
grep -E "passed|failed" $OUT/pytest_lsd.log | tail -1
timeout -k 10 120 python3 tools/bench_group.py 1310720 12500000 > $OUT/bench_group.log 2>&1 || { echo BG_FAIL; exit 1; }
cut -c1-160 $OUT/bench_group.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $OUT/pmc -o run --output-format csv -- python3 $R/tools/bench_group.py 12500000 > $OUT/pmc.log 2>&1 || { echo PMC_FAIL; exit 1; }
echo LSD_OK
