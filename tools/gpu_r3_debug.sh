#!/bin/bash
# Round 3: the GPU suite against the debug build (libsd_hip_cas_debug.so: the device-side
# conservation checks of csrc/sd_debug.h on every multi-round LDS kernel).  A test after
# which the violation counter moved fails (tests/conftest.py).  Usage: gpu_r3_debug.sh <tag> [k expr]
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r3_debug}
mkdir -p $OUT
cd $R
export SD_HIP_CAS_LIB=$R/spacedrive_amd/libsd_hip_cas_debug.so SD_CAS_DEBUG_INVARIANTS=1
K=${2:-}
timeout -k 10 1100 python3 -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 600 --timeout-method thread ${K:+-k "$K"} > $OUT/pytest_gpu_debug.log 2>&1 || { echo PYTEST_FAIL; tail -40 $OUT/pytest_gpu_debug.log; exit 1; }
tail -3 $OUT/pytest_gpu_debug.log
grep -c "SD_CAS invariant" $OUT/pytest_gpu_debug.log || true
