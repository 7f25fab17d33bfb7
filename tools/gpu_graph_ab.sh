#!/bin/bash
# hipGraph A/B for the grouping launch sequence: GPU grouping tests (graphs on), then the
# bench's serial group timing and bench_group with and without graphs (interleaved).
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/graph
mkdir -p $OUT
cd $R
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 250 --timeout-method thread -k "group or shard or multi or bench_scale or identifier or headline" > $OUT/pytest.log 2>&1 || { echo PYTEST_FAIL; exit 1; }
for r in 1 2; do
  SD_CAS_NO_GRAPHS=1 timeout -k 10 300 python3 -u tools/bench_group.py > $OUT/nograph_$r.log 2>&1 || { echo NG_FAIL; exit 1; }
  timeout -k 10 300 python3 -u tools/bench_group.py > $OUT/graph_$r.log 2>&1 || { echo G_FAIL; exit 1; }
done
timeout -k 10 300 python3 -u bench.py --steps 5 --no-cpu-baseline > $OUT/bench.log 2>&1 || { echo BENCH_FAIL; exit 1; }
echo GRAPH_OK
