#!/bin/bash
# Round 3: A/B of K1 variants (tools/ablib/libsd_hip_cas_*.so built by tools/build_variant.sh) against
# the in-tree build, interleaved 3 rounds, 1,310,720 files, keys digest compared.  Usage: <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r3_abk1}
mkdir -p $OUT
cd $R
for round in 1 2 3; do
  for lib in current $R/tools/ablib/libsd_hip_cas_*.so; do
    name=$(basename $lib .so)
    if [ $lib = current ]; then unset SD_HIP_CAS_LIB; else export SD_HIP_CAS_LIB=$lib; fi
    timeout -k 10 200 python3 -u tools/prof_sampled.py --files 1310720 --iters 6 > $OUT/time_${name}_r$round.log 2>&1 || { echo "TIME_FAIL $name"; tail -5 $OUT/time_${name}_r$round.log; exit 1; }
    echo "$name r$round $(grep -o '[0-9.]* ms' $OUT/time_${name}_r$round.log | tail -5 | tr '\n' ' ') $(grep keys_digest $OUT/time_${name}_r$round.log)"
  done
done
echo ABK1_OK
