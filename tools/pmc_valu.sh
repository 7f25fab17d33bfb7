#!/bin/bash
# Round 4: VALU-busy PMC pass (one rocprofv3 --pmc run per workload, --kernel-trace only):
# K1G and K1 at the bench's 1.31M files, K2 on config 2 (1M whole files), the validator's small and
# docs shapes.  SQ 6 + GRBM 2 counters per pass.  Usage: pmc_valu.sh <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r4_pmc_valu}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
C="SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT"
i=0
for cmd in "$R/tools/prof_sampled.py --files 1310720 --iters 2 --fused" "$R/tools/prof_sampled.py --files 1310720 --iters 2" "$R/tools/prof_k2.py --iters 2" "$R/tools/prof_checksums.py --shape small --shape docs --iters 2"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $C -d $OUT/p$i -o run --output-format csv -- python3 $cmd > $OUT/p$i.log 2>&1 || { echo "PMC pass $i failed ($cmd)"; tail -5 $OUT/p$i.log; exit 1; }
  tail -2 $OUT/p$i.log
done
python3 $R/tools/pmc_valu.py $OUT > $OUT/valu.json && cat $OUT/valu.json
echo PMC_VALU_OK
