#!/bin/bash
# Fused-chain region-count A/B: the fused GPU tests on the in-tree library, then the bench's
# K1G and fused-table numbers for the in-tree library and for tools/ablib/$2.so (alternating).
set -euo pipefail
OUT=gpurun_out/$1
VAR=$2
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests -x -v --timeout 120 --timeout-method thread -m gpu \
  -k "fused or regions" > "$OUT/pytest_gpu.log" 2>&1
tail -1 "$OUT/pytest_gpu.log"
for r in 1 2; do
  timeout -k 10 240 python3 -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --sustain-seconds 0 \
    --e2e-files 0 > "$OUT/bench_cur_r$r.json" 2> "$OUT/bench_cur_r$r.err"
  SD_HIP_CAS_LIB=$PWD/tools/ablib/$VAR.so timeout -k 10 240 python3 -u bench.py --steps 10 --warmup 3 \
    --no-cpu-baseline --sustain-seconds 0 --e2e-files 0 > "$OUT/bench_var_r$r.json" 2> "$OUT/bench_var_r$r.err"
done
python3 - "$OUT" <<'PY'
import json, sys, glob, os
for f in sorted(glob.glob(sys.argv[1] + "/bench_*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    fu = d.get("group", {}).get("fused", {})
    print(os.path.basename(f), d["value"], d["roofline"].get("kernel_ms"), {k: fu.get(k) for k in fu if "ms" in k})
PY
echo REG_OK
