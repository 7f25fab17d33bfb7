#!/bin/bash
# Multi-GPU code paths on a one-GPU box: the fixed-capacity exchange kernels and the
# multi-device creation (pytest), then bench.py's N=2 rehearsal (2 ranks on one GPU, gloo).
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-multi}
mkdir -p $OUT
cd $R
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -k "fixed_capacity or multi_device or sharded" > $OUT/pytest_multi.log 2>&1 || { echo PYTEST_FAIL; tail -30 $OUT/pytest_multi.log; exit 1; }
export SD_BENCH_ONE_DEVICE=1
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 --files-per-gpu 131072 --no-cpu-baseline --sustain-seconds 0 --e2e-files 262144 > $OUT/bench_n2.log 2>&1 || { echo N2_FAIL; tail -30 $OUT/bench_n2.log; exit 1; }
tail -1 $OUT/bench_n2.log
echo MULTI_OK
