#!/bin/bash
# Round-end evidence pass: parity suite, smoke, headline bench (local and exchange path),
# other BASELINE configs, rocprofv3 kernel stats of the bench command, PMC passes on K1.
# Each GPU step has its own time limit; stop at the first failure.
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/final
mkdir -p $OUT
cd $R
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; exit 1; }
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo SMOKE_FAIL; exit 1; }
timeout -k 10 400 python3 -u bench.py > $OUT/bench.log 2>&1 || { echo BENCH_FAIL; exit 1; }
timeout -k 10 400 python3 -u bench.py --exchange --no-cpu-baseline > $OUT/bench_exchange.log 2>&1 || { echo BENCHX_FAIL; exit 1; }
timeout -k 10 900 python3 -u tools/bench_configs.py --config 2 --config 3e --config 4 --config 5 --config 1 > $OUT/configs.log 2>&1 || { echo CONFIGS_FAIL; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o bench --output-format csv -- python3 $R/bench.py --steps 5 --warmup 1 --no-cpu-baseline > $OUT/bench_prof.log 2>&1 || { echo PROF_FAIL; exit 1; }
i=0
for grp in "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE" "SQ_INSTS_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES" "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_ACTIVE_INST_ANY" "GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $grp -d $OUT/pmc/p$i -o run --output-format csv -- python3 $R/tools/prof_sampled.py --iters 2 > $OUT/pmc_p$i.log 2>&1 || { echo "PMC_FAIL $i"; exit 1; }
done
echo FINAL_OK
