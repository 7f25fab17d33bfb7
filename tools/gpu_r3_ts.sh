#!/bin/bash
# Round 3: sd_bucket_min per-workgroup phase timing (tools/ts_bucket_min.py) for every
# tools/ablib/ts_*.so (ts_big*: the big tables at 1.31 M keys; others: the fine tables at
# 12.5 M and 100 M keys).  Usage: <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r3_ts}
mkdir -p $OUT
cd $R
for lib in $R/tools/ablib/ts_*.so; do
  name=$(basename $lib .so)
  case $name in ts_big*) sizes="1310720";; *) sizes="12500000 100000000";; esac
  for n in $sizes; do
    SD_HIP_CAS_LIB=$lib timeout -k 10 200 python3 -u tools/ts_bucket_min.py $n > $OUT/${name}_$n.log 2>&1 || { echo "FAIL $name"; tail -5 $OUT/${name}_$n.log; exit 1; }
    echo "== $name $n"; tail -1 $OUT/${name}_$n.log | cut -c1-420
  done
done
echo TS_OK
