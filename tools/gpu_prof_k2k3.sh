#!/bin/bash
# rocprofv3 evidence for the config-2 (K2, ragged whole files) and config-5 (K3, 64 GiB
# checksum) kernels: kernel-trace stats, then PMC passes (HBM bytes, VALU issue), each in
# its own run.  Stops at the first failure.
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/k2k3
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/k2_stats -o run --output-format csv -- python3 $R/tools/prof_packed.py > $OUT/k2_stats.log 2>&1 || { echo K2_STATS_FAIL; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/k3_stats -o run --output-format csv -- python3 $R/tools/prof_checksum.py --iters 5 > $OUT/k3_stats.log 2>&1 || { echo K3_STATS_FAIL; exit 1; }
i=0
for grp in "FETCH_SIZE" "SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $grp -d $OUT/pmc_k2/p$i -o run --output-format csv -- python3 $R/tools/prof_packed.py > $OUT/pmc_k2_p$i.log 2>&1 || { echo "PMC_K2_FAIL $i"; exit 1; }
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $grp -d $OUT/pmc_k3/p$i -o run --output-format csv -- python3 $R/tools/prof_checksum.py --iters 2 > $OUT/pmc_k3_p$i.log 2>&1 || { echo "PMC_K3_FAIL $i"; exit 1; }
done
echo K2K3_OK
