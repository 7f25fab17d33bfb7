#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
for f in 1250000 1245184 1310720 1250000 1310720; do
  echo "files=$f $(timeout -k 10 200 python3 -u tools/prof_sampled.py --files $f --iters 4 2>/dev/null | grep 'iter 3')" >> gpurun_out/tail.log || exit 1
done
