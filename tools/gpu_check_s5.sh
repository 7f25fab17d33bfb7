set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/s5
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/s5/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; exit 1; }
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s5/smoke.log 2>&1 || { echo SMOKE_FAIL; exit 1; }
timeout -k 10 400 python3 -u bench.py > gpurun_out/s5/bench.log 2>&1 || { echo BENCH_FAIL; exit 1; }
echo ALL_OK
