#!/bin/bash
# rocprofv3 kernel stats: grouping at the bench's 1.31M keys, and config 2 (K2).
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/prof2
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/grp -o grp --output-format csv -- python3 $R/tools/bench_group.py 1310720 > $OUT/grp.log 2>&1 || { echo GRP_FAIL; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/k2 -o k2 --output-format csv -- python3 $R/tools/bench_configs.py --config 2 > $OUT/k2.log 2>&1 || { echo K2_FAIL; exit 1; }
echo PROF2_OK
