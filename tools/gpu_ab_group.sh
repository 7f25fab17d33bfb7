#!/bin/bash
# Interleaved grouping timings of A/B builds: gpu_ab_group.sh <tag> <lib names in tools/ablib>...
# ("cur" = the in-tree build).  Parity of the in-tree build is the pytest pass.
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=$1; shift
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
for i in 1 2 3; do
  for L in "$@"; do
    if [ "$L" = cur ]; then LIB=""; else LIB=$R/tools/ablib/$L.so; fi
    SD_HIP_CAS_LIB=$LIB timeout -k 10 120 python3 tools/bench_group.py 1310720 12500000 > $OUT/${L}_$i.log 2>&1 || { echo "FAIL $L"; cat $OUT/${L}_$i.log; exit 1; }
    python3 -c "
import json,sys
r=[json.loads(l) for l in open('$OUT/${L}_$i.log') if l.startswith('{')]
print('$L', ' '.join('%d:%.4f' % (x['keys'], x['hash_group_ms']) for x in r), 'identical' if all(x['identical'] for x in r) else 'MISMATCH')"
  done
done
echo AB_OK
