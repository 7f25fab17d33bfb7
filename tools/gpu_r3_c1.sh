#!/bin/bash
# Round 3: config 1 (10k tmpfs files through sd_cas_generate_cas_ids_from_paths) x3 and the
# from_paths GPU tests.  Usage: <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r3_c1}
mkdir -p $OUT
cd $R
timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 200 --timeout-method thread -k "from_paths or example or identifier_job" > $OUT/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for r in 1 2 3; do
  timeout -k 10 300 python3 -u tools/bench_configs.py --config 1 > $OUT/c1_$r.log 2>&1 || { echo C1_FAIL; tail -20 $OUT/c1_$r.log; exit 1; }
  grep '^{' $OUT/c1_$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('gpu', round(d['gpu_dropin_files_per_s']), 'cpu', round(d['cpu_oracle_all_cores_simd_files_per_s']), 'step100', d['job_step_100_ms'], d['parity'])"
done
