#!/bin/bash
# Occupancy A/B of the lane-per-file kernels (the validator lane kernel ran fastest at 2
# waves/SIMD): K1 at 4 (in-tree) / 3 / 2 waves per SIMD, K2 at 4 / 3 / 2, by unused dynamic
# LDS at launch (tools/ablib/patch_k1occ*.py, patch_k2occ*.py); interleaved twice.
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r2b_occ_ab}
mkdir -p $OUT
cd $R
for round in 1 2; do
  for v in intree k1occ3 k1occ2; do
    if [ $v = intree ]; then L=""; else L=$R/tools/ablib/$v.so; fi
    SD_HIP_CAS_LIB=$L timeout -k 10 180 python3 -u tools/prof_sampled.py --files 1310720 --iters 6 > $OUT/k1.$v.$round.log 2>&1 || { echo FAIL $v; tail -20 $OUT/k1.$v.$round.log; exit 1; }
    echo "== K1 $v round $round: $(tail -3 $OUT/k1.$v.$round.log | tr '\n' ' ')"
  done
  for v in intree k2occ3 k2occ2; do
    if [ $v = intree ]; then L=""; else L=$R/tools/ablib/$v.so; fi
    SD_HIP_CAS_LIB=$L timeout -k 10 180 python3 -u tools/prof_packed.py > $OUT/k2.$v.$round.log 2>&1 || { echo FAIL $v; tail -20 $OUT/k2.$v.$round.log; exit 1; }
    echo "== K2 $v round $round: $(head -2 $OUT/k2.$v.$round.log | tr '\n' ' ')"
  done
done
