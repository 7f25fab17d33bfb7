#!/bin/bash
# rocprofv3 kernel-trace stats of the headline bench command, then one FETCH_SIZE pass on K1.
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/profb
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o bench --output-format csv -- python3 $R/bench.py --steps 5 --warmup 1 --no-cpu-baseline > $OUT/bench_prof.log 2>&1 || { echo PROF_FAIL; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $OUT/pmc -o run --output-format csv -- python3 $R/tools/prof_sampled.py --iters 2 > $OUT/pmc.log 2>&1 || { echo PMC_FAIL; exit 1; }
echo PROFB_OK
