#!/bin/bash
# streamed file_checksum A/B of builds (tools/ab_file_checksum.py), interleaved x2
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-fcab}; shift
mkdir -p $OUT
cd $R
for i in 1 2; do
  for L in "$@"; do
    if [ "$L" = cur ]; then LIB=""; else LIB=$R/tools/ablib/$L.so; fi
    SD_HIP_CAS_LIB=$LIB timeout -k 10 240 python3 tools/ab_file_checksum.py > $OUT/${L}_$i.log 2>&1 || { echo "FAIL $L"; tail -5 $OUT/${L}_$i.log; exit 1; }
    echo "$L $(grep '^{' $OUT/${L}_$i.log)"
  done
done
echo FCAB_OK
