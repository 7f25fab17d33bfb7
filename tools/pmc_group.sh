#!/bin/bash
# PMC passes (separate rocprofv3 runs, counters + kernel trace only) over the grouping
# kernels at 12.5M keys: HBM-side bytes per kernel (FETCH_SIZE x2 per the gfx950 note in
# MI355X_MICROARCH.md, WRITE_SIZE) and L2 hit rate.
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/pmcg
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc $grp -d $OUT/p$i -o run --output-format csv -- python3 $R/tools/bench_group.py 12500000 > $OUT/p$i.log 2>&1 || { echo "PMC pass $i ($grp) failed"; exit 1; }
done
echo PMCG_OK
