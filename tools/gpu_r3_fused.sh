#!/bin/bash
# Round 3: the fused hash + group chain — its GPU tests, the A/B timing (tools/prof_fused.py),
# and a check that the debug build's invariant counter fires (a variant whose downsweep check
# is deliberately off by one must fail a sort test).  Usage: gpu_r3_fused.sh <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r3_fused}
mkdir -p $OUT
cd $R
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -k "fused" > $OUT/pytest_fused.log 2>&1 || { echo PYTEST_FAIL; tail -40 $OUT/pytest_fused.log; exit 1; }
tail -1 $OUT/pytest_fused.log
timeout -k 10 300 python3 -u tools/prof_fused.py > $OUT/prof_fused.log 2>&1 || { echo PROF_FAIL; tail -20 $OUT/prof_fused.log; exit 1; }
tail -1 $OUT/prof_fused.log
if [ -f tools/ablib/dbg_inject.so ]; then
  SD_HIP_CAS_LIB=$R/tools/ablib/dbg_inject.so SD_CAS_DEBUG_INVARIANTS=1 timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread -k "test_sort_pairs_vs_numpy" > $OUT/pytest_inject.log 2>&1; rc=$?
  echo "injected-violation run rc=$rc (expected 1)"; grep -m2 "SD_CAS invariant\|device invariant" $OUT/pytest_inject.log
fi
echo FUSED_DONE
