#!/bin/bash
# Round 3: A/B of grouping-chain variants (tools/ablib/libsd_hip_cas_g_*.so) against the
# in-tree build, interleaved 2 rounds, 12.5 M and 100 M keys (tools/ab_group.py).  Usage: <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r3_abg}
mkdir -p $OUT
cd $R
for round in 1 2; do
  for lib in current $R/tools/ablib/libsd_hip_cas_g_*.so; do
    name=$(basename $lib .so)
    if [ $lib = current ]; then unset SD_HIP_CAS_LIB; else export SD_HIP_CAS_LIB=$lib; fi
    timeout -k 10 200 python3 -u tools/ab_group.py 12500000 100000000 > $OUT/g_${name}_r$round.log 2>&1 || { echo "FAIL $name"; tail -5 $OUT/g_${name}_r$round.log; exit 1; }
    tail -1 $OUT/g_${name}_r$round.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['lib'], 'r$round', {k: (round(v['ms'],4), round(v['hbm_frac'],3), v['rep_digest']) for k, v in d.items() if k != 'lib'})"
  done
done
echo ABG_OK
