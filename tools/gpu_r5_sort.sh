#!/bin/bash
# Round 5 LSD sort rework (wave-private scatter + row scan): the sort / grouping parity tests
# on the release and debug libraries, the 12.5 M-key chain timing, a kernel trace and the
# PMC bytes-per-key passes (tools/gpu_r5_pmc_sort.sh).  Usage: gpu_r5_sort.sh <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r5_sort}
mkdir -p $OUT
cd $R
K="sort_pairs or group_vs_oracle or group_methods or group_min_vs or identifier_links or lane or checksums or packed"
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "$K" > $OUT/pytest.log 2>&1 || { echo TEST_FAIL; tail -20 $OUT/pytest.log; exit 1; }
tail -n 1 $OUT/pytest.log
SD_HIP_CAS_LIB=$R/spacedrive_amd/libsd_hip_cas_debug.so SD_CAS_DEBUG_INVARIANTS=1 timeout -k 10 400 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "sort_pairs or group_methods or group_min_vs or identifier_links" > $OUT/pytest_debug.log 2>&1 || { echo DEBUG_FAIL; tail -20 $OUT/pytest_debug.log; exit 1; }
tail -n 1 $OUT/pytest_debug.log
timeout -k 10 120 python3 tools/bench_group.py 1310720 12500000 > $OUT/bench_group.log 2>&1 || { echo BG_FAIL; tail -5 $OUT/bench_group.log; exit 1; }
grep keys $OUT/bench_group.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 $R/tools/bench_group.py --only lsd 12500000 > $OUT/prof.log 2>&1 || { echo PROF_FAIL; exit 1; }
cd $R
bash tools/gpu_r5_pmc_sort.sh ${1:-r5_sort}/pmc
