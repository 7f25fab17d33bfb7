#!/bin/bash
# Round 4: interleaved A/B of library builds: for round in 1 2, for every tools/ablib/*.so and
# the in-tree build, run each given tool command (SD_HIP_CAS_LIB selects the build).
# Usage: gpu_r4_ab.sh <tag> <cmd>...
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r4_ab}
shift
mkdir -p $OUT
cd $R
for round in $(seq 1 ${AB_ROUNDS:-2}); do
  for lib in $R/tools/ablib/*.so current; do
    name=$(basename $lib .so)
    if [ $lib = current ]; then unset SD_HIP_CAS_LIB; else export SD_HIP_CAS_LIB=$lib; fi
    i=0
    for cmd in "$@"; do
      i=$((i+1))
      echo "== $name r$round: $cmd" >> $OUT/ab.log
      timeout -k 10 300 bash -c "$cmd" >> $OUT/ab.log 2>&1 || { echo "AB_FAIL $name $cmd"; tail -5 $OUT/ab.log; exit 1; }
    done
    echo "$name r$round done"
  done
done
unset SD_HIP_CAS_LIB
echo AB_OK
