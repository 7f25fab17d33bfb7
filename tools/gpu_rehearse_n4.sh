#!/bin/bash
# Rehearsal of bench.py's multi-rank path with 2 and 4 ranks sharing the one GPU of a
# gpurun box (exchange over gloo): correctness of the N > 1 code path, not a scaling number.
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/n4
mkdir -p $OUT
cd $R
export SD_BENCH_ONE_DEVICE=1
for n in 2 4; do
  timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port 2953$n bench.py --gpus $n --steps 3 --warmup 1 --files-per-gpu 131072 --no-cpu-baseline > $OUT/bench_n$n.log 2>&1 || { echo N${n}_FAIL; exit 1; }
done
echo N4_OK
