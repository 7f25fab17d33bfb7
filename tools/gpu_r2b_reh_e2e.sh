#!/bin/bash
# N=2 rehearsal of bench.py incl. the e2e and sustained legs (two ranks on one GPU over gloo).
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-reh_e2e}
mkdir -p $OUT
cd $R
export SD_BENCH_ONE_DEVICE=1
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29561 bench.py --gpus 2 --steps 3 --warmup 1 --files-per-gpu 131072 --no-cpu-baseline --e2e-files 262144 --sustain-seconds 1 > $OUT/bench_n2.log 2>&1 || { echo "N2_FAIL"; tail -20 $OUT/bench_n2.log; exit 1; }
grep '^{' $OUT/bench_n2.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('N', d['n_gpus'], 'value', d['value'], 'e2e', d['e2e'], 'sustained', d['sustained'])"
