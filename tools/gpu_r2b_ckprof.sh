#!/bin/bash
# Batched validator timing (device shapes + tmpfs paths) and its rocprofv3 kernel stats.
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r2b_ckprof}
mkdir -p $OUT
cd $R
timeout -k 10 400 python3 -u tools/prof_checksums.py --paths 2000 > $OUT/checksums.log 2>&1 || { echo CK_FAIL; tail -20 $OUT/checksums.log; exit 1; }
timeout -k 10 200 python3 -u tools/prof_checksum.py --gib 16 --iters 5 >> $OUT/checksums.log 2>&1 || { echo K3_FAIL; exit 1; }
cat $OUT/checksums.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o ck --output-format csv -- python3 $R/tools/prof_checksums.py --shape photos --shape small --iters 3 > $OUT/ck_prof.log 2>&1 || { echo PROF_FAIL; tail -20 $OUT/ck_prof.log; exit 1; }
find $OUT/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $OUT/ck_kernel_stats.csv
head -12 $OUT/ck_kernel_stats.csv
