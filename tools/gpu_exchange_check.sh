#!/bin/bash
# Exchange path checks: RCCL world-1 parity test, bench --exchange (world 1), 2/4-rank rehearsal.
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/xchk
mkdir -p $OUT
cd $R
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 250 --timeout-method thread -k "rccl or shard" > $OUT/pytest.log 2>&1 || { echo PYTEST_FAIL; exit 1; }
for r in 1 2; do
timeout -k 10 300 python3 -u bench.py --exchange --no-cpu-baseline > $OUT/exch_$r.log 2>&1 || { echo X_FAIL; exit 1; }
done
export SD_BENCH_ONE_DEVICE=1
for n in 2 4; do
  timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port 2954$n bench.py --gpus $n --steps 3 --warmup 1 --files-per-gpu 131072 --no-cpu-baseline > $OUT/bench_n$n.log 2>&1 || { echo N${n}_FAIL; exit 1; }
done
echo XCHK_OK
