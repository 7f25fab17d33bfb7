#!/bin/bash
# 100-file job-step A/B of builds (tools/prof_jobstep.py), interleaved x2
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-jsab}; shift
mkdir -p $OUT
cd $R
for i in 1 2; do
  for L in "$@"; do
    if [ "$L" = cur ]; then LIB=""; else LIB=$R/tools/ablib/$L.so; fi
    SD_HIP_CAS_LIB=$LIB timeout -k 10 200 python3 tools/prof_jobstep.py > $OUT/${L}_$i.log 2>&1 || { echo "FAIL $L"; tail -5 $OUT/${L}_$i.log; exit 1; }
    echo "$L $(grep -h 'median' $OUT/${L}_$i.log | tr '\n' ' ')"
  done
done
echo JSAB_OK
