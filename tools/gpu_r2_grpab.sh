#!/bin/bash
# Grouping A/B: parity tests on the new build, then interleaved timings of the previous
# build (tools/ablib/lib_group_v0.so) and the new one at 1.31M and 12.5M keys.
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-grpab}
mkdir -p $OUT
cd $R
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -k "group or partition or sharded or multi or identifier or workspace or config4 or headline or bench_scale or fixed" > $OUT/pytest_group.log 2>&1 || { echo PYTEST_FAIL; tail -40 $OUT/pytest_group.log; exit 1; }
grep -E "passed|failed" $OUT/pytest_group.log | tail -1
for i in 1 2; do
  SD_HIP_CAS_LIB=$R/tools/ablib/lib_group_v0.so timeout -k 10 120 python3 tools/bench_group.py 1310720 12500000 > $OUT/old_$i.log 2>&1 || { echo OLD_FAIL; exit 1; }
  timeout -k 10 120 python3 tools/bench_group.py 1310720 12500000 > $OUT/new_$i.log 2>&1 || { echo NEW_FAIL; cat $OUT/new_$i.log; exit 1; }
  echo "old $i"; grep keys $OUT/old_$i.log | cut -c1-120
  echo "new $i"; grep keys $OUT/new_$i.log | cut -c1-120
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace -o grp -- python3 $R/tools/bench_group.py 1310720 12500000 > $OUT/trace.log 2>&1 || { echo TRACE_FAIL; exit 1; }
echo GRPAB_OK
