#!/bin/bash
# Grouping evidence: grid-barrier vs launch-gap microbenchmark, then per-dispatch kernel
# trace of the hash grouping at the bench size (1.31M keys) and config 4's share (12.5M).
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-gprof}
mkdir -p $OUT
cd $R
timeout -k 10 60 ./tools/ubench_gridsync > $OUT/ubench_gridsync.log 2>&1 || { echo UBENCH_FAIL; cat $OUT/ubench_gridsync.log; exit 1; }
cat $OUT/ubench_gridsync.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace -o grp -- python3 $R/tools/bench_group.py 1310720 12500000 > $OUT/bench_group.log 2>&1 || { echo TRACE_FAIL; tail $OUT/bench_group.log; exit 1; }
cat $OUT/bench_group.log | grep keys
echo GPROF_OK
