#!/bin/bash
# Grouping changes: parity tests (grouping / sort / config 4 / multi-device) + kernel split at 12.5M and 1.31M keys.
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r2b_grp}
mkdir -p $OUT
cd $R
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -k "group or sort_pairs or config4 or multi_device or exchange or links or sharded" > $OUT/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
cd /tmp && export TMPDIR=/tmp
for n in 12500000 1310720; do
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/prof$n -o g --output-format csv -- python3 $R/tools/bench_group.py $n > $OUT/log$n 2>&1 || { echo PROF_FAIL; tail $OUT/log$n; exit 1; }
grep hash_group_ms $OUT/log$n | cut -c1-200
find $OUT/prof$n -name "*kernel_stats.csv" -exec grep -E "sd_part|sd_bucket|Name" {} \;
done
