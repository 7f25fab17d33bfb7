#!/bin/bash
# PMC passes for K1 (separate rocprofv3 runs, counters only with --kernel-trace; no sys/runtime trace)
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/pmc
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "SQ_INSTS_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES" "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_ACTIVE_INST_ANY" "GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $grp -d $OUT/p$i -o run --output-format csv -- python3 $R/tools/prof_sampled.py --files ${FILES:-1250000} --iters 2 > $OUT/p$i.log 2>&1 || { echo "PMC pass $i ($grp) failed"; exit 1; }
done
echo PMC_OK
