#!/bin/bash
# K2 packing-alignment A/B (128-B synth packing vs 16-B packed contents): timing twice, then one
# FETCH_SIZE pass for the HBM bytes of each layout.  Stops at the first failure.
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/k2align
mkdir -p $OUT
cd $R
for r in 1 2; do
  timeout -k 10 300 python3 -u tools/prof_packed.py >> $OUT/ab.log 2>&1 || { echo TIME_FAIL; exit 1; }
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $OUT/pmc -o run --output-format csv -- python3 $R/tools/prof_packed.py > $OUT/pmc.log 2>&1 || { echo PMC_FAIL; exit 1; }
echo K2ALIGN_OK
