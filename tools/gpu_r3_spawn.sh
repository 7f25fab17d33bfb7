#!/bin/bash
# Round 3: bench.py --gpus N launches its own ranks.  (1) --gpus 2 rehearsal with both ranks
# on the box's one GPU (SD_BENCH_ONE_DEVICE=1, exchange over gloo): one JSON line, n_gpus 2,
# non-null exchange; (2) plain --gpus 2 on a one-GPU box must exit non-zero; (3) --gpus 1.
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r3_spawn}
mkdir -p $OUT
cd $R
SD_BENCH_ONE_DEVICE=1 timeout -k 10 400 python3 -u bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu-baseline --e2e-files 0 --sustain-seconds 0 > $OUT/bench_n2_rehearsal.log 2>&1 || { echo REH_FAIL; tail -30 $OUT/bench_n2_rehearsal.log; exit 1; }
grep -c '^{' $OUT/bench_n2_rehearsal.log
grep '^{' $OUT/bench_n2_rehearsal.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('n_gpus', d['n_gpus'], 'value', d['value'], 'k1', d['roofline']['kernel_ms_ranks'], 'exchange', d['config']['exchange'])"
timeout -k 10 200 python3 -u bench.py --gpus 2 --steps 2 --warmup 1 > $OUT/bench_n2_nodev.log 2>&1; rc=$?
echo "plain --gpus 2 rc=$rc"; tail -2 $OUT/bench_n2_nodev.log
[ $rc -ne 0 ] || { echo NODEV_NOT_REFUSED; exit 1; }
timeout -k 10 300 python3 -u bench.py --gpus 1 --steps 5 --warmup 1 --no-cpu-baseline --e2e-files 0 --sustain-seconds 0 > $OUT/bench_n1.log 2>&1 || { echo N1_FAIL; tail -20 $OUT/bench_n1.log; exit 1; }
tail -1 $OUT/bench_n1.log | cut -c1-300
echo SPAWN_OK
