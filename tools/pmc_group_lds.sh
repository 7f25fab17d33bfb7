#!/bin/bash
# PMC passes over the grouping chain at 12.5 M keys (tools/bench_group.py): LDS traffic,
# bank conflicts, LDS issue stalls and wave state per kernel.  One counter group per
# rocprofv3 run (kernel trace + counters only).  Usage: <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-pmcg_lds}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES" "SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" "GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $grp -d $OUT/p$i -o run --output-format csv -- python3 $R/tools/bench_group.py 12500000 > $OUT/p$i.log 2>&1 || { echo "PMC pass $i ($grp) failed"; tail -5 $OUT/p$i.log; exit 1; }
done
python3 $R/tools/pmc_summarize.py $OUT > $OUT/summary.json
python3 - $OUT/summary.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
for k, v in d.items():
    if k.startswith("sd_"):
        print(k[:40], {c: round(x) for c, x in v.items()})
PY
echo PMCG_LDS_OK
