#!/bin/bash
# A/B of the bench step pipeline on one GPU: local grouping vs the RCCL key-range
# exchange path (world 1), with the grouping issued inline (host syncs stall the next
# K1 enqueue) or from the worker thread; then the 2-rank rehearsal (gloo, one device).
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/xab
mkdir -p $OUT
cd $R
B="python3 -u bench.py --steps 10 --warmup 2 --no-cpu-baseline"
timeout -k 10 300 $B > $OUT/local.log 2>&1 || { echo LOCAL_FAIL; exit 1; }
timeout -k 10 300 $B --exchange --inline-group > $OUT/exch_inline.log 2>&1 || { echo INLINE_FAIL; exit 1; }
timeout -k 10 300 $B --exchange > $OUT/exch_thread.log 2>&1 || { echo THREAD_FAIL; exit 1; }
timeout -k 10 300 $B --inline-group > $OUT/local_inline.log 2>&1 || { echo LI_FAIL; exit 1; }
export SD_BENCH_ONE_DEVICE=1
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 --files-per-gpu 131072 --no-cpu-baseline > $OUT/bench_n2.log 2>&1 || { echo N2_FAIL; exit 1; }
echo XAB_OK
