#!/bin/bash
# Rehearsal of bench.py's N > 1 path (fixed-capacity key-range exchange) with 2 and 4 ranks
# sharing the one GPU of a gpurun box over gloo: correctness of the code path, not scaling.
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-reh2}
mkdir -p $OUT
cd $R
export SD_BENCH_ONE_DEVICE=1
for N in 2 4; do
  timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 --master-port $((29540 + N)) bench.py --gpus $N --steps 3 --warmup 1 --files-per-gpu 131072 --no-cpu-baseline --e2e-files 0 --sustain-seconds 0 > $OUT/bench_n$N.log 2>&1 || { echo "N${N}_FAIL"; tail -20 $OUT/bench_n$N.log; exit 1; }
  grep '^{' $OUT/bench_n$N.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('N', d['n_gpus'], 'value', d['value'], 'exchange', d['config'].get('exchange'))"
done
echo REH_OK
