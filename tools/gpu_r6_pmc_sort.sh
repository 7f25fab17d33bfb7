#!/bin/bash
# Round 6 (round 5: VERDICT r4 #5): HBM bytes per key of the default hash grouping and the forced LSD
# sort at 12.5 M keys — one process per method (tools/bench_group.py --only), one rocprofv3
# --pmc pass per counter group (FETCH_SIZE, WRITE_SIZE, TCC hit/miss), then tools/pmc_sort.py.
# Usage: gpu_r6_pmc_sort.sh <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r6_pmc_sort}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for m in hash lsd lsdapi; do
  for g in "fetch:FETCH_SIZE" "write:WRITE_SIZE" "hit:TCC_HIT_sum TCC_MISS_sum"; do
    tag=${g%%:*}; c=${g#*:}
    timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $c -d $OUT/${m}_$tag -o run --output-format csv -- python3 $R/tools/bench_group.py --only $m 12500000 > $OUT/${m}_$tag.log 2>&1 || { echo "PMC $m $tag failed"; tail -5 $OUT/${m}_$tag.log; exit 1; }
  done
done
python3 $R/tools/pmc_sort.py $OUT > $OUT/pmc_sort.json && python3 -c "import json;d=json.load(open('$OUT/pmc_sort.json'));print({m:(round(d[m]['measured_b_per_key'],1),d[m]['algorithmic_b_per_key']) for m in d if m in ('hash','lsd','lsdapi')})"
echo PMC_SORT_OK
