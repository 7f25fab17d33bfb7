#!/bin/bash
# Round-4 evidence pass: GPU suite, smoke, headline bench (fused chain at N=1), the --gpus 2
# one-device rehearsal, BASELINE configs 1-4, the validator shapes, rocprofv3 kernel stats of
# the bench, PMC passes on K1G (HBM bytes) and the VALU-busy pass.  Usage: <tag> [skip-suite]
# Each GPU step has its own time limit; stop at the first failure.
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r4_final}
mkdir -p $OUT
cd $R
if [ -z "$2" ]; then
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -30 $OUT/pytest_gpu.log; exit 1; }
  tail -1 $OUT/pytest_gpu.log
  timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo SMOKE_FAIL; exit 1; }
fi
timeout -k 10 400 python3 -u bench.py > $OUT/bench.log 2>&1 || { echo BENCH_FAIL; tail -20 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log | cut -c1-300
SD_BENCH_ONE_DEVICE=1 timeout -k 10 400 python3 -u bench.py --gpus 2 --steps 5 --warmup 1 --sustain-seconds 0 --e2e-files 1048576 > $OUT/bench_n2_rehearsal.log 2>&1 || { echo REH_FAIL; tail -20 $OUT/bench_n2_rehearsal.log; exit 1; }
timeout -k 10 600 python3 -u tools/bench_configs.py --config 2 --config 3e --config 4 --config 1 > $OUT/configs.log 2>&1 || { echo CONFIGS_FAIL; tail -20 $OUT/configs.log; exit 1; }
timeout -k 10 300 python3 -u tools/prof_checksums.py --paths 2000 > $OUT/validator.log 2>&1 || { echo VALIDATOR_FAIL; tail -20 $OUT/validator.log; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o bench --output-format csv -- python3 $R/bench.py --steps 5 --warmup 1 --no-cpu-baseline --sustain-seconds 0 --e2e-files 0 > $OUT/bench_prof.log 2>&1 || { echo PROF_FAIL; exit 1; }
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 200 rocprofv3 --kernel-trace --pmc $grp -d $OUT/pmc/p$i -o run --output-format csv -- python3 $R/tools/prof_sampled.py --files 1310720 --iters 2 --fused > $OUT/pmc_p$i.log 2>&1 || { echo "PMC_FAIL $i ($grp)"; exit 1; }
done
bash $R/tools/pmc_valu.sh ${1:-r4_final}/pmc_valu > $OUT/pmc_valu_run.log 2>&1 || { echo PMC_VALU_FAIL; tail -5 $OUT/pmc_valu_run.log; exit 1; }
echo FINAL_OK
