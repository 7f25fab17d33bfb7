#!/bin/bash
# LSD sort A/B of builds (tools/ab_sort.py and the sort path of tools/bench_group.py), x2
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
for i in 1 2; do
  for L in "$@"; do
    if [ "$L" = cur ]; then LIB=""; else LIB=$R/tools/ablib/$L.so; fi
    SD_HIP_CAS_LIB=$LIB timeout -k 10 200 python3 tools/ab_sort.py 2>&1 | grep "^{" | sed "s/^/$L /" || exit 1
    SD_HIP_CAS_LIB=$LIB timeout -k 10 200 python3 tools/bench_group.py 2>&1 | grep "^{" | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print('$L', 'keys', d['keys'], 'lsd_group_ms', round(d['lsd_group_ms'],4), 'hash_ms', round(d['hash_group_ms'],4), d['identical'])" || exit 1
  done
done
echo SORTAB_OK
