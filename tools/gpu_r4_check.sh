#!/bin/bash
# Round 4: a GPU test subset, then optional tool runs given as extra args (each its own
# time limit).  Usage: gpu_r4_check.sh <tag> '<k expr>' [tool command]...
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r4_check}
mkdir -p $OUT
cd $R
K=$2
shift 2
if [ -n "$K" ]; then
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -k "$K" > $OUT/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -40 $OUT/pytest_gpu.log; exit 1; }
  tail -1 $OUT/pytest_gpu.log
fi
i=0
for cmd in "$@"; do
  i=$((i+1))
  echo "== $cmd" > $OUT/tool$i.log
  timeout -k 10 400 bash -c "$cmd" >> $OUT/tool$i.log 2>&1 || { echo "TOOL_FAIL $i: $cmd"; tail -20 $OUT/tool$i.log; exit 1; }
  tail -4 $OUT/tool$i.log
done
echo CHECK_OK
