#!/bin/bash
# BASELINE configs 1-5 on one GPU (tools/bench_configs.py), one JSON line each.
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/cfg
mkdir -p $OUT
cd $R
timeout -k 10 900 python3 -u tools/bench_configs.py ${CONFIGS:---config 2 --config 3e --config 4 --config 5 --config 1} > $OUT/configs.log 2>&1 || { echo CONFIGS_FAIL; exit 1; }
echo CONFIGS_OK
