#!/bin/bash
# A/B: K1 v1 (ab/libsd_hip_cas_v1.so) vs current, then GPU tests on current, then PMC of both.
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/ab
mkdir -p $OUT
cd $R
SD_HIP_CAS_LIB=$R/ab/libsd_hip_cas_v1.so timeout -k 10 300 python3 -u tools/prof_sampled.py --iters 4 > $OUT/time_v1.log 2>&1 || { echo V1_FAIL; exit 1; }
timeout -k 10 300 python3 -u tools/prof_sampled.py --iters 4 > $OUT/time_v2.log 2>&1 || { echo V2_FAIL; exit 1; }
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; exit 1; }
cd /tmp && export TMPDIR=/tmp
for v in v1 v2; do
  if [ $v = v1 ]; then export SD_HIP_CAS_LIB=$R/ab/libsd_hip_cas_v1.so; else unset SD_HIP_CAS_LIB; fi
  i=0
  for grp in "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum" "SQ_INSTS_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES" "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_ACTIVE_INST_ANY" "GRBM_GUI_ACTIVE"; do
    i=$((i+1))
    timeout -k 10 300 rocprofv3 --kernel-trace --pmc $grp -d $OUT/pmc_$v/p$i -o run --output-format csv -- python3 $R/tools/prof_sampled.py --iters 2 > $OUT/pmc_${v}_p$i.log 2>&1 || { echo "PMC $v pass $i failed"; exit 1; }
  done
done
echo AB_OK
