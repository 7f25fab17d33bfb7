#!/bin/bash
# A/B: 2,048-slot tables in 256-lane workgroups (SD_GROUP_SMALL_TABLES=1, mean bucket 768)
# (the SD_GROUP_SMALL_TABLES knob and sd_bucket_min_small were removed after this A/B)
# vs 4,096-slot tables in 512-lane workgroups (mean 1,536), interleaved.
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r2b_sab}
mkdir -p $OUT
cd $R
for rep in 1 2 3; do
for k in 0 1; do
  for n in 12500000 4000000; do
  SD_GROUP_SMALL_TABLES=$k timeout -k 10 120 python3 tools/bench_group.py $n > $OUT/s$k.$n.$rep.log 2>&1 || { echo FAIL $k; tail $OUT/s$k.$n.$rep.log; exit 1; }
  echo "small=$k n=$n rep=$rep $(grep -o '"hash_group_ms": [0-9.]*' $OUT/s$k.$n.$rep.log) $(grep -o '"identical": [a-z]*' $OUT/s$k.$n.$rep.log)"
  done
done
done
