#!/bin/bash
# Round-6 evidence pass, in three gpurun calls (each fits one call's time limit):
#   suite   GPU suite on the release library, then on the debug build (device-side invariant
#           checks, csrc/sd_debug.h), smoke
#   bench   headline bench (fused chain at N=1, live rocm-smi power in the line), rocprofv3
#           --kernel-trace --stats of the bench, PMC passes on K1G (HBM bytes), the --gpus 2 / 4
#           / 8 one-GPU rehearsals (checked by tools/rehearsal_check.py)
#   extra   BASELINE configs 1-4, the validator shapes and file path, link emission, randomised
#           stress (grouping with the forced LSD path every iteration, the fused chain, link
#           emission vs the replay, the path gather + validator file path vs the C oracle)
# Usage: gpu_r6_final.sh <tag> suite|bench|extra.  Each GPU step has its own time limit; the
# script stops at the first failure.
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r6_final}
mkdir -p $OUT
cd $R
case "$2" in
suite)
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -30 $OUT/pytest_gpu.log; exit 1; }
  tail -1 $OUT/pytest_gpu.log
  SD_HIP_CAS_LIB=$R/spacedrive_amd/libsd_hip_cas_debug.so SD_CAS_DEBUG_INVARIANTS=1 timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 600 --timeout-method thread > $OUT/pytest_gpu_debug.log 2>&1 || { echo DEBUG_FAIL; tail -30 $OUT/pytest_gpu_debug.log; exit 1; }
  tail -1 $OUT/pytest_gpu_debug.log
  timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo SMOKE_FAIL; exit 1; }
  tail -1 $OUT/smoke.log
  echo SUITE_OK ;;
bench)
  timeout -k 10 400 python3 -u bench.py --steps 20 --warmup 3 > $OUT/bench.log 2>&1 || { echo BENCH_FAIL; tail -20 $OUT/bench.log; exit 1; }
  tail -1 $OUT/bench.log | cut -c1-300
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o bench --output-format csv -- python3 $R/bench.py --steps 5 --warmup 1 --no-cpu-baseline --sustain-seconds 0 --e2e-files 0 > $OUT/bench_prof.log 2>&1) || { echo PROF_FAIL; exit 1; }
  i=0
  for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
    i=$((i+1))
    (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 200 rocprofv3 --kernel-trace --pmc $grp -d $OUT/pmc/p$i -o run --output-format csv -- python3 $R/tools/prof_sampled.py --files 1310720 --iters 2 --fused > $OUT/pmc_p$i.log 2>&1) || { echo "PMC_FAIL $i ($grp)"; exit 1; }
  done
  python3 $R/tools/pmc_summarize.py $OUT/pmc > $OUT/pmc_k1g.json
  SD_BENCH_ONE_DEVICE=1 SD_CPU_BASELINE_THREADS=16 timeout -k 10 500 python3 -u bench.py --gpus 2 --steps 10 --warmup 2 --files-per-gpu 262144 --e2e-files 1048576 > $OUT/bench_n2_rehearsal.log 2>&1 || { echo REH2_FAIL; tail -20 $OUT/bench_n2_rehearsal.log; exit 1; }
  SD_BENCH_ONE_DEVICE=1 SD_CPU_BASELINE_THREADS=16 timeout -k 10 500 python3 -u bench.py --gpus 4 --steps 10 --warmup 2 --files-per-gpu 131072 --e2e-files 1048576 > $OUT/bench_n4_rehearsal.log 2>&1 || { echo REH4_FAIL; tail -20 $OUT/bench_n4_rehearsal.log; exit 1; }
  SD_BENCH_ONE_DEVICE=1 SD_CPU_BASELINE_THREADS=16 timeout -k 10 500 python3 -u bench.py --gpus 8 --steps 10 --warmup 2 --files-per-gpu 65536 --e2e-files 524288 > $OUT/bench_n8_rehearsal.log 2>&1 || { echo REH8_FAIL; tail -20 $OUT/bench_n8_rehearsal.log; exit 1; }
  for n in 2 4 8; do python3 tools/rehearsal_check.py $OUT/bench_n${n}_rehearsal.log $n || { echo "REH${n}_CHECK_FAIL"; exit 1; }; done
  echo BENCH_OK ;;
extra)
  SD_CONFIG1_PASSES=7 timeout -k 10 600 python3 -u tools/bench_configs.py --config 2 --config 3e --config 4 --config 1 > $OUT/configs.log 2>&1 || { echo CONFIGS_FAIL; tail -20 $OUT/configs.log; exit 1; }
  timeout -k 10 300 python3 -u tools/prof_checksums.py --paths 2000 --path-runs 6 > $OUT/validator.log 2>&1 || { echo VALIDATOR_FAIL; tail -20 $OUT/validator.log; exit 1; }
  timeout -k 10 300 python3 -u tools/prof_links.py > $OUT/links.log 2>&1 || { echo LINKS_FAIL; tail -20 $OUT/links.log; exit 1; }
  timeout -k 10 240 python3 -u tools/stress_parity.py --seconds 120 --lsd-every 1 > $OUT/stress_parity_lsd.log 2>&1 || { echo STRESS_FAIL; tail -5 $OUT/stress_parity_lsd.log; exit 1; }
  timeout -k 10 200 python3 -u tools/stress_parity.py --seconds 60 --fused > $OUT/stress_fused.log 2>&1 || { echo STRESS_FAIL; tail -5 $OUT/stress_fused.log; exit 1; }
  timeout -k 10 200 python3 -u tools/stress_links.py --seconds 60 > $OUT/stress_links.log 2>&1 || { echo STRESS_FAIL; tail -5 $OUT/stress_links.log; exit 1; }
  timeout -k 10 200 python3 -u tools/stress_paths.py --checksums --seconds 60 > $OUT/stress_paths.log 2>&1 || { echo STRESS_FAIL; tail -5 $OUT/stress_paths.log; exit 1; }
  for f in stress_parity_lsd stress_fused stress_links stress_paths; do tail -1 $OUT/$f.log | cut -c1-200; done
  echo EXTRA_OK ;;
*) echo "usage: gpu_r6_final.sh <tag> suite|bench|extra"; exit 2 ;;
esac
