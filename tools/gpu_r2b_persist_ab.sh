#!/bin/bash
# A/B of sd_bucket_min's grid: one workgroup per bucket (0) vs k workgroups per CU walking them.
# (the SD_GROUP_PERSIST knob and sd_bucket_min_pf were removed after this A/B: profiles/r02b_bucket_min_persist_ab.log)
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r2b_pab}
mkdir -p $OUT
cd $R
for rep in 1 2; do
for k in 0 3 4 6 12; do
  SD_GROUP_PERSIST=$k timeout -k 10 120 python3 tools/bench_group.py 12500000 > $OUT/p$k.$rep.log 2>&1 || { echo FAIL $k; tail $OUT/p$k.$rep.log; exit 1; }
  echo "persist=$k rep=$rep $(grep -o '"hash_group_ms": [0-9.]*' $OUT/p$k.$rep.log) $(grep -o '"identical": [a-z]*' $OUT/p$k.$rep.log)"
done
done
