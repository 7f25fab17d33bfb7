#!/bin/bash
# Rehearsal of bench.py's multi-rank path (RCCL key-range exchange) with 2 ranks sharing
# the one GPU of a gpurun box: correctness of the N > 1 code path, not a scaling number.
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/n2
mkdir -p $OUT
cd $R
export SD_BENCH_ONE_DEVICE=1
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 --files-per-gpu 131072 --no-cpu-baseline > $OUT/bench_n2.log 2>&1 || { echo N2_FAIL; exit 1; }
echo N2_OK
