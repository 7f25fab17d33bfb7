#!/bin/bash
# Round 3: per-kernel ablation of the grouping chain at 12.5 M keys.  For the in-tree build
# and every tools/ablib/abl_*.so (timing-only patches from tools/ab_patches/), the chain's
# median ms (tools/ab_group.py) and a rocprofv3 --kernel-trace --stats table.  Usage: <tag> [n]
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r3_abl}
N=${2:-12500000}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for lib in current $R/tools/ablib/abl_*.so; do
  name=$(basename $lib .so)
  if [ $lib = current ]; then unset SD_HIP_CAS_LIB; else export SD_HIP_CAS_LIB=$lib; fi
  timeout -k 10 200 python3 -u $R/tools/ab_group.py $N > $OUT/t_$name.log 2>&1 || { echo "FAIL $name"; tail -5 $OUT/t_$name.log; exit 1; }
  tail -1 $OUT/t_$name.log | cut -c1-200
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/prof_$name -o run --output-format csv -- python3 $R/tools/ab_group.py $N > $OUT/p_$name.log 2>&1 || { echo "PROF_FAIL $name"; exit 1; }
  f=$(find $OUT/prof_$name -name 'run_kernel_stats.csv' | head -1)
  echo "== $name"; cut -d, -f1-4 $f | head -8
done
echo ABL_OK
