#!/bin/bash
# Validator lane-per-buffer path: checksum GPU tests, then the batch shapes with the
# in-tree library (lane path from 65,536 buffers, <= 128 chunks, 3 waves/SIMD) against
# variants without it, at 2 waves/SIMD, and for <= 64 chunks (tools/ablib/patch_*.py).
# (Passes: 1 = in-tree <= 64 chunks from 131,072 buffers vs nolane / lane128 / lanemin16k;
# 2 = the defaults above; 3 = VARIANTS='intree laneocc2 laneocc1 lane512' on the big shapes;
# 4 = the tail cut: VARIANTS='intree nolane lanenocut lanetail1' with the skewed shapes.
# (First pass: in-tree = <= 64 chunks from 131,072 buffers vs nolane / lane128 / lanemin16k.)
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r2b_lane_ab}
mkdir -p $OUT
cd $R
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -k "checksum" > $OUT/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
SH=${SH:-"--shape small16k --shape small32k --shape small64k --shape small128k --shape small256k --shape small --shape docs64 --shape docs --iters 5"}
for round in 1 2; do
  for v in ${VARIANTS:-intree nolane laneocc2 lane64}; do
    if [ $v = intree ]; then L=""; else L=$R/tools/ablib/$v.so; fi
    SD_HIP_CAS_LIB=$L timeout -k 10 240 python3 -u tools/prof_checksums.py $SH > $OUT/$v.$round.log 2>&1 || { echo FAIL $v; tail -20 $OUT/$v.$round.log; exit 1; }
    echo "== $v round $round"; python3 -c "
import json,sys
for l in open('$OUT/$v.$round.log'):
    if l.startswith('{'):
        d=json.loads(l); print(f\"{d['shape']:10s} {d['ms']:8.3f} ms {d['gb_per_s']/1e3:6.3f} TB/s {d['buffers_per_s']/1e6:7.1f} M/s parity={d['parity']}\")
"
  done
done
