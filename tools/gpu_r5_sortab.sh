#!/bin/bash
# A/B of the LSD sort scatter (round 5): parity tests, then the wave-private scatter vs the
# round-2 downsweep (SD_CAS_SORT_LEGACY=1) at 1.31 M and 12.5 M keys, then a kernel-trace.
set -o pipefail
mkdir -p gpurun_out/sortab
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "sort_pairs or group_vs_oracle or group_methods or group_min_vs or identifier_links" > gpurun_out/sortab/pytest.log 2>&1
SD_HIP_CAS_LIB=$PWD/spacedrive_amd/libsd_hip_cas_debug.so SD_CAS_DEBUG_INVARIANTS=1 timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "sort_pairs or group_methods or group_min_vs" > gpurun_out/sortab/pytest_debug.log 2>&1
for i in 1 2; do
SD_CAS_SORT_LEGACY=1 timeout -k 10 120 python3 tools/bench_group.py --only lsd 1310720 12500000 >> gpurun_out/sortab/legacy.log 2>&1
SD_CAS_SORT_LEGACY=0 timeout -k 10 120 python3 tools/bench_group.py --only lsd 1310720 12500000 >> gpurun_out/sortab/new.log 2>&1
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/sortab/prof -o run -- python3 tools/bench_group.py --only lsd 12500000 > gpurun_out/sortab/prof.log 2>&1
