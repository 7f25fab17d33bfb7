#!/bin/bash
# Round 3: grouping-table rework.  (1) the grouping GPU tests on the in-tree build, (2) the
# chain at 1.31 M / 12.5 M / 100 M keys: in-tree vs every tools/ablib/g_*.so, interleaved 2
# rounds (tools/ab_group.py), (3) rocprofv3 kernel stats of the in-tree chain at 12.5 M.
# Usage: <tag>   (env SIZES = key counts, PROF=0 skips (3))
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r3_abg2}
mkdir -p $OUT
cd $R
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -k "group or sort or fused or region or exchange or links or config4 or sharded or multi_device" > $OUT/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
for round in 1 2; do
  for lib in current $R/tools/ablib/g_*.so; do
    name=$(basename $lib .so)
    if [ $lib = current ]; then unset SD_HIP_CAS_LIB; else export SD_HIP_CAS_LIB=$lib; fi
    timeout -k 10 200 python3 -u tools/ab_group.py ${SIZES:-1310720 12500000 100000000} > $OUT/g_${name}_r$round.log 2>&1 || { echo "FAIL $name"; tail -5 $OUT/g_${name}_r$round.log; exit 1; }
    tail -1 $OUT/g_${name}_r$round.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['lib'], 'r$round', {k: (round(v['ms'],4), round(v['hbm_frac'],3), v['objects'], v['rep_digest']) for k, v in d.items() if k != 'lib'})"
  done
done
[ "${PROF:-1}" = 0 ] && { echo ABG2_OK; exit 0; }
cd /tmp && export TMPDIR=/tmp
for lib in current $R/tools/ablib/g_*.so; do
  name=$(basename $lib .so)
  if [ $lib = current ]; then unset SD_HIP_CAS_LIB; else export SD_HIP_CAS_LIB=$lib; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/prof_$name -o run --output-format csv -- python3 $R/tools/ab_group.py ${PROFN:-12500000} > $OUT/prof_$name.log 2>&1 || { echo "PROF_FAIL $name"; exit 1; }
  f=$(find $OUT/prof_$name -name 'run_kernel_stats.csv' | head -1)
  echo "== $name"; grep '"sd_' $f | cut -d, -f1-4
done
echo ABG2_OK
