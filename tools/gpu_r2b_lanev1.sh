#!/bin/bash
# Same-box A/B of the validator chain: in-tree (tail cut, sorted class ranges) vs the first
# lane-path version (tools/ablib/patch_lanev1.py), then a rocprofv3 kernel-stats pass of
# the in-tree chain on the 1 M small-buffer shape.
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r2b_lanev1}
mkdir -p $OUT
cd $R
for round in 1 2; do
  for v in intree lanev1; do
    if [ $v = intree ]; then L=""; else L=$R/tools/ablib/$v.so; fi
    SD_HIP_CAS_LIB=$L timeout -k 10 200 python3 -u tools/prof_checksums.py ${SH:---shape small --shape small256k --shape docs --shape skew1m --iters 5} > $OUT/$v.$round.log 2>&1 || { echo FAIL $v; tail -20 $OUT/$v.$round.log; exit 1; }
    echo "== $v round $round"; grep "^{" $OUT/$v.$round.log | cut -c1-90
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o small --output-format csv -- python3 $R/tools/prof_checksums.py --shape small --iters 3 > $OUT/prof.log 2>&1 || { echo PROF_FAIL; exit 1; }
find $OUT/prof -name "*kernel_stats.csv" -exec cut -d, -f1-4 {} \; | head -20
