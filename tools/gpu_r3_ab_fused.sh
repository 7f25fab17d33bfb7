#!/bin/bash
# Round 3: GPU suite, then the headline bench fused (default) vs --unfused, interleaved x2,
# rocprofv3 kernel stats of the fused bench, and PMC passes on K1G.  Usage: <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r3_abf}
mkdir -p $OUT
cd $R
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
for r in 1 2; do
  timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --e2e-files 0 --sustain-seconds 0 --steps 20 --warmup 3 > $OUT/bench_fused_$r.log 2>&1 || { echo BENCH_FAIL; tail -20 $OUT/bench_fused_$r.log; exit 1; }
  timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --e2e-files 0 --sustain-seconds 0 --steps 20 --warmup 3 --unfused > $OUT/bench_unfused_$r.log 2>&1 || { echo BENCH_FAIL; tail -20 $OUT/bench_unfused_$r.log; exit 1; }
  for m in fused unfused; do
    tail -1 $OUT/bench_${m}_$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); g=d['config']; r=d['roofline']; gr=d['group'] or {}; print('$m', round(d['value']/1e6,2), 'M/s step', round(d['ms_per_step'],3), 'kern', round(r['kernel_ms'],3), 'frac', round(r['frac'],4), 'group.ms', gr.get('ms'), 'fused', (gr.get('fused') or {}).get('tables_ms'), (gr.get('fused') or {}).get('parity_vs_standalone'))"
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o bench --output-format csv -- python3 $R/bench.py --steps 5 --warmup 1 --no-cpu-baseline --sustain-seconds 0 --e2e-files 0 > $OUT/bench_prof.log 2>&1 || { echo PROF_FAIL; exit 1; }
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "SQ_INSTS_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES" "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_ACTIVE_INST_ANY" "GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -k 10 200 rocprofv3 --kernel-trace --pmc $grp -d $OUT/pmc/p$i -o run --output-format csv -- python3 $R/tools/prof_sampled.py --files 1310720 --iters 2 --fused > $OUT/pmc_p$i.log 2>&1 || { echo "PMC_FAIL $i ($grp)"; exit 1; }
done
echo ABF_OK
