#!/bin/bash
# grouping on adversarial key sets (tools/ab_group_adversarial.py) for A/B builds, x2
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
for i in 1 2; do
  for L in "$@"; do
    if [ "$L" = cur ]; then LIB=""; else LIB=$R/tools/ablib/$L.so; fi
    SD_HIP_CAS_LIB=$LIB timeout -k 10 200 python3 tools/ab_group_adversarial.py 2>&1 | grep "^{" | sed "s/^/$L /" || exit 1
  done
done
