#!/bin/bash
# Round 5: the VALU / power evidence of K1 and K1G in ONE gpurun session:
# compute-only ceiling (tools/ubench_k1, built in-tree beforehand), rocm-smi clock probe, and
# one rocprofv3 --pmc pass per kernel; combined by tools/valu_power.py.
# Usage: gpu_r5_valu_power.sh <tag> <session id>
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r5_valu_power}
mkdir -p $OUT
timeout -k 10 120 $R/tools/ubench_k1 > $OUT/ubench_k1.log 2>&1 || { echo "ubench_k1 failed"; tail -5 $OUT/ubench_k1.log; exit 1; }
tail -12 $OUT/ubench_k1.log
(cd $R && timeout -k 10 240 python3 tools/clock_probe.py --seconds 6 k1 k1c k1g > $OUT/clock.jsonl 2> $OUT/clock.err) || { echo "clock_probe failed"; tail -5 $OUT/clock.err; exit 1; }
cat $OUT/clock.jsonl
cd /tmp && export TMPDIR=/tmp
C="SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT"
i=0
for cmd in "$R/tools/prof_sampled.py --files 1310720 --iters 2 --fused" "$R/tools/prof_sampled.py --files 1310720 --iters 2"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $C -d $OUT/p$i -o run --output-format csv -- python3 $cmd > $OUT/p$i.log 2>&1 || { echo "PMC pass $i failed ($cmd)"; tail -5 $OUT/p$i.log; exit 1; }
  tail -2 $OUT/p$i.log
done
python3 $R/tools/valu_power.py $OUT "$2" > $OUT/r05_valu_power.json && head -40 $OUT/r05_valu_power.json
echo VALU_POWER_OK
