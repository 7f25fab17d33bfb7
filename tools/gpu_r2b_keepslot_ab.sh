#!/bin/bash
# A/B: refine prefetch only (abl/lib_refine_pf.so) vs + totals/scatter prefetch (abl/lib_all_pf.so), interleaved.
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r2b_ksab}
mkdir -p $OUT
cd $R
for rep in 1 2 3; do
for L in lib_cur lib_keepslot; do
  for n in 12500000 1310720; do
  SD_HIP_CAS_LIB=$R/abl/$L.so timeout -k 10 120 python3 tools/bench_group.py $n > $OUT/$L.$n.$rep.log 2>&1 || { echo FAIL $L; tail $OUT/$L.$n.$rep.log; exit 1; }
  echo "$L n=$n rep=$rep $(grep -o '"hash_group_ms": [0-9.]*' $OUT/$L.$n.$rep.log) $(grep -o '"identical": [a-z]*' $OUT/$L.$n.$rep.log)"
  done
done
done
