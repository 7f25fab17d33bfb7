#!/bin/bash
# (the SD_GROUP_BIG_TARGET knob was removed after this A/B: profiles/r02b_group_big_tables_ab.log)
# A/B: refine into 12,288-slot tables (SD_GROUP_BIG_TARGET=3072) vs the 4,096-slot plan
# vs 4,096-slot tables in 512-lane workgroups (mean 1,536), interleaved.
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r2b_bab}
mkdir -p $OUT
cd $R
for rep in 1 2 3; do
for k in 0 3072; do
  for n in 12500000 4000000; do
  SD_GROUP_BIG_TARGET=$k timeout -k 10 120 python3 tools/bench_group.py $n > $OUT/s$k.$n.$rep.log 2>&1 || { echo FAIL $k; tail $OUT/s$k.$n.$rep.log; exit 1; }
  echo "bigtarget=$k n=$n rep=$rep $(grep -o '"hash_group_ms": [0-9.]*' $OUT/s$k.$n.$rep.log) $(grep -o '"identical": [a-z]*' $OUT/s$k.$n.$rep.log)"
  done
done
done
