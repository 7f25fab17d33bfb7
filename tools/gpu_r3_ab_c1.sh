#!/bin/bash
# Round 3: A/B of the from_paths gather windows (tools/ablib/libsd_hip_cas_c1_*.so vs the
# in-tree build) on BASELINE config 1's 10k tmpfs files, interleaved 3 rounds.  Usage: <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r3_abc1}
mkdir -p $OUT
cd $R
D=/dev/shm/sdcas_c1_$$
python3 - "$D" > $OUT/list.txt <<'PY'
import math, os, sys
import numpy as np
d = sys.argv[1]; os.makedirs(d, exist_ok=True)
rng = np.random.default_rng(1)
sizes = np.exp(rng.uniform(math.log(1024), math.log(10 * 1024 * 1024), 10000)).astype(np.int64)
for i, s in enumerate(sizes):
    p = f"{d}/f{i:05d}"
    with open(p, "wb") as fh:
        fh.write(rng.integers(0, 256, int(s), dtype=np.uint8).tobytes())
    print(p, int(s))
PY
for round in 1 2 3; do
  for lib in current $R/tools/ablib/libsd_hip_cas_c1_*.so; do
    if [ $lib = current ]; then unset SD_HIP_CAS_LIB; else export SD_HIP_CAS_LIB=$lib; fi
    timeout -k 10 200 python3 -u tools/ab_c1.py $OUT/list.txt > $OUT/t_$(basename $lib .so)_r$round.log 2>&1 || { echo FAIL; tail -5 $OUT/t_$(basename $lib .so)_r$round.log; rm -rf $D; exit 1; }
    tail -1 $OUT/t_$(basename $lib .so)_r$round.log
  done
done
rm -rf $D
