#!/bin/bash
# Round 4: the full GPU suite on the release library, then again on the debug library
# (device-side invariant checks of csrc/sd_debug.h).  Usage: gpu_r4_suite.sh <tag> [k expr]
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r4_suite}
mkdir -p $OUT
cd $R
K=${2:-}
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread ${K:+-k "$K"} > $OUT/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
[ -n "$SKIP_DEBUG" ] && exit 0
SD_HIP_CAS_LIB=$R/spacedrive_amd/libsd_hip_cas_debug.so SD_CAS_DEBUG_INVARIANTS=1 timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 600 --timeout-method thread ${K:+-k "$K"} > $OUT/pytest_gpu_debug.log 2>&1 || { echo DEBUG_FAIL; tail -40 $OUT/pytest_gpu_debug.log; exit 1; }
tail -1 $OUT/pytest_gpu_debug.log
echo SUITE_OK
