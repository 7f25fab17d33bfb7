#!/bin/bash
# Round 3: identifier-links job timing (tools/prof_links.py) and its rocprofv3 kernel stats.
# Usage: <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r3_links}
mkdir -p $OUT
cd $R
timeout -k 10 300 python3 -u tools/prof_links.py > $OUT/links_timing.log 2>&1 || { echo LINKS_FAIL; tail -5 $OUT/links_timing.log; exit 1; }
cat $OUT/links_timing.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 $R/tools/prof_links.py > $OUT/prof.log 2>&1 || { echo PROF_FAIL; exit 1; }
f=$(find $OUT/prof -name 'run_kernel_stats.csv' | head -1)
cut -d, -f1-4 $f | head -14
echo LINKS_OK
