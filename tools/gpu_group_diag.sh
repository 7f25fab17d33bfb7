#!/bin/bash
# Where does sd_bucket_min_big spend its time at 1.31M keys?  rocprofv3 kernel stats of
# bench_group.py under diagnosis variants (tools/ablib/patch_g{b,c,d}.py; results wrong by design).
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/gdiag
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for L in ${LIBS:-cur lib_diag_gb lib_diag_gc lib_diag_gd}; do
  if [ "$L" = cur ]; then LIB=""; else LIB=$R/tools/ablib/$L.so; fi
  SD_HIP_CAS_LIB=$LIB timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/$L -o k --output-format csv -- python3 $R/tools/bench_group.py 1310720 > $OUT/$L.log 2>&1 || { echo "FAIL $L"; tail -5 $OUT/$L.log; exit 1; }
  echo "== $L"; grep -E '"sd_(bucket|part)' $OUT/$L/k_kernel_stats.csv | cut -d, -f1-4
done
echo GDIAG_OK
